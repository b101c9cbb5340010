# Round 4: multi-rank plan + tile-pair list reuse -- parity (sharded vs one
# rank, bitwise) and the per-rank kernel chain at global1m R=8, reuse off / on.
set -u
OUT=gpurun_out/r4h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread \
    tests/test_gpu_multirank.py tests/test_gpu_tile_reuse.py tests/test_gpu_sim.py \
    > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for A in 0 1; do
  BSA_TPR=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/probe_tpr$A -o run --output-format csv -- \
      python tools/probe_rank.py global1m 8 2 20 > $OUT/probe_tpr$A.log 2>&1
  rc=$?; echo "probe tpr=$A rc=$rc"; tail -2 $OUT/probe_tpr$A.log; [ $rc -eq 0 ] || exit $rc
done
BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_trace.so BSA_PF_TRACE_FILE=$OUT/pf_trace.bin timeout -k 10 200 \
    python tools/pf_trace.py run box100k > $OUT/pf_trace_run.log 2>&1 && python tools/pf_trace.py show $OUT/pf_trace.bin > $OUT/pf_trace.txt 2>&1
rc=$?; echo "trace rc=$rc"; tail -12 $OUT/pf_trace.txt
for L in libbsaccel.so libbsaccel_k2r256l2.so libbsaccel.so libbsaccel_k2r256l2.so; do
  BSACCEL_LIB=$PWD/bluesky_amd/$L timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$L.json 2> $OUT/bench_$L.err || { tail -3 $OUT/bench_$L.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$L.json'))
print('$L ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
done
BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_k2r256l2.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_k2 -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > $OUT/prof_k2.log 2>&1; echo "prof rc=$?"
