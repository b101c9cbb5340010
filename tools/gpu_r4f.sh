# Round 4, pass f: tile-pair list reuse budget A/B on the headline bench.
set -u
OUT=gpurun_out/r4f
mkdir -p $OUT
for V in 0:0 1:500 1:1000 1:2016 0:0 1:500 1:1000 1:2016; do
  T=${V%%:*}; S=${V##*:}
  BSA_TPR=$T BSA_TPR_SH=$S timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_${T}_${S}.json 2> $OUT/bench.err || { tail -3 $OUT/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_${T}_${S}.json'))
print('tpr $T sh $S ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()}, d['tile_reuse_rank0']['builds'], d['tile_reuse_rank0']['detects'])"
done
for L in libbsaccel.so libbsaccel_k2l1.so libbsaccel.so libbsaccel_k2l1.so; do
  BSACCEL_LIB=$PWD/bluesky_amd/$L timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$L.json 2> $OUT/bench.err || { tail -3 $OUT/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$L.json'))
print('$L ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sim.py tests/test_gpu_tile_reuse.py tests/test_gpu_multirank.py tests/test_gpu_trace.py -m gpu -k "not 8ranks and not key_blocks" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $OUT/pytest.log
BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_stamps.so timeout -k 10 120 python tools/stamps.py > $OUT/stamps.log 2>&1; echo "stamps rc=$?"; tail -4 $OUT/stamps.log
