# Prefilter iteration on the GPU: detect + sim + fullsize parity, the headline
# bench, the per-rank probe and the item timelines (trace build).
set -u
TAG=${TAG:-pf}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_detect.py tests/test_gpu_fullsize.py tests/test_gpu_sim.py tests/test_gpu_multirank.py tests/test_gpu_reuse.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print('ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
timeout -k 10 300 python tools/rowslice_probe.py > $OUT/rowslice.log 2>&1
rc=$?; cat $OUT/rowslice.log; [ $rc -eq 0 ] || exit $rc
export BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_trace.so
for a in "box100k 1" "box100k 8" "global1m 1"; do
  set -- $a
  BSA_PF_TRACE_FILE=$OUT/tr.bin timeout -k 10 120 python tools/pf_trace.py run $1 $2 || exit 1
  echo "== trace $1 R=$2"; python tools/pf_trace.py show $OUT/tr.bin | grep -v "detect 1" | head -8
  rm -f $OUT/tr.bin
done
