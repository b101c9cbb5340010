# Round 4: heavy items first (prefilter load balance) + K0d fused -- parity,
# then A/B's of the bench (fused K0d on / off, heavy on / off, near pieces 8)
# and the kernel stats of the fused / separate K0d builds.
set -u
OUT=gpurun_out/r4m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread \
    tests/test_gpu_tile_reuse.py tests/test_gpu_multirank.py tests/test_gpu_sim.py tests/test_gpu_detect.py \
    > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; grep "builds" $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag env...
  local T=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$T.json 2> $OUT/bench_$T.err || { tail -3 $OUT/bench_$T.err; return 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$T.json'))
print('$T ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
}
for i in 1 2; do
  run f0h0_$i BSA_K0D_FUSE=0 BSA_PF_HEAVY=0 || exit 1
  run f0h1_$i BSA_K0D_FUSE=0 BSA_PF_HEAVY=1 || exit 1
  run f1h1_$i BSA_K0D_FUSE=1 BSA_PF_HEAVY=1 || exit 1
  run f0h1u6_$i BSA_K0D_FUSE=0 BSA_PF_HEAVY=1 BSA_PF_HEAVY_US=6 || exit 1
  run f0h0pn8_$i BSA_K0D_FUSE=0 BSA_PF_HEAVY=0 BSA_PF_PIECES_NEAR=8 || exit 1
done
for F in 1 0; do
  BSA_K0D_FUSE=$F timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/prof_f$F -o run --output-format csv -- \
      python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/prof_f$F.log 2>&1; rc=$?; echo "prof fuse=$F rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - <<PY
import csv, glob
f = glob.glob('$OUT/prof_f$F/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]:
    print('fuse=$F %-34s calls %4s avg %8.2f us total %9.1f us' % (r['Name'][:34], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e3))
PY
  find $OUT/prof_f$F -name "*kernel_trace.csv" -size +4M -delete
done
