# Round 4: multi-rank plan reuse + K0d fused into the prefilter -- parity,
# the per-rank chain at global1m R=8 (plan reuse off / on), the prefilter's
# item timeline, and A/B's: K0d fused / separate, K2 256 rows x 2 lanes, K1b grid.
set -u
OUT=gpurun_out/r4j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread \
    tests/test_gpu_tile_reuse.py tests/test_gpu_multirank.py tests/test_gpu_sim.py tests/test_gpu_detect.py \
    > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; grep "builds" $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for A in 0 1; do
  BSA_TPR=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/probe_tpr$A -o run --output-format csv -- \
      python tools/probe_rank.py global1m 8 2 20 > $OUT/probe_tpr$A.log 2>&1
  rc=$?; echo "probe tpr=$A rc=$rc"; tail -1 $OUT/probe_tpr$A.log; [ $rc -eq 0 ] || exit $rc
done
run() {  # tag lib env...
  local T=$1 L=$2; shift 2
  env BSACCEL_LIB=$PWD/bluesky_amd/$L "$@" timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$T.json 2> $OUT/bench_$T.err || { tail -3 $OUT/bench_$T.err; return 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$T.json'))
print('$T ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()}, d.get('tile_reuse_rank0', {}).get('builds'))"
}
for i in 1 2; do
  run fuse1_$i libbsaccel.so BSA_K0D_FUSE=1 || exit 1
  run fuse0_$i libbsaccel.so BSA_K0D_FUSE=0 || exit 1
  run k2v_$i libbsaccel_k2r256l2.so BSA_K0D_FUSE=1 || exit 1
  run k1b768_$i libbsaccel.so BSA_K1B_GRID=768 || exit 1
done
BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_trace.so BSA_PF_TRACE_FILE=$OUT/pf_trace.bin timeout -k 10 200 \
    python tools/pf_trace.py run box100k > $OUT/pf_trace_run.log 2>&1 && python tools/pf_trace.py show $OUT/pf_trace.bin > $OUT/pf_trace.txt 2>&1
rc=$?; echo "trace rc=$rc"; tail -12 $OUT/pf_trace.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python bench.py --steps 40 --warmup 3 --no-cpu --no-variants > $OUT/prof.log 2>&1; echo "prof rc=$?"
