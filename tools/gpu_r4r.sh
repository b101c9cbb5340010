# K2 fused with K4' (one rank; alt / vs / gse / gsn double-buffered): parity
# of the resident step, then A/B (BSA_K24=0 / 1, same build)
set -u
OUT=gpurun_out/r4r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_sim.py tests/test_gpu_tile_reuse.py tests/test_gpu_trace.py tests/test_gpu_asas_dropin.py tests/test_gpu_feed.py tests/test_gpu_mvp_kin.py \
    tests/test_gpu_multirank.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" $OUT/tests.log | head -20; exit $rc; }
run() {  # tag env...
  local T=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$T.json 2> $OUT/bench_$T.err || { tail -3 $OUT/bench_$T.err; return 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$T.json'))
print('$T ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
}
for i in 1 2 3; do
  run k24off_$i BSA_K24=0 || exit 1
  run k24on_$i BSA_K24=1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python bench.py --steps 40 --warmup 3 --no-cpu --no-variants > $OUT/prof.log 2>&1; echo "prof rc=$?"
python - <<PY
import csv, glob
f = glob.glob('$OUT/prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print('%-34s calls %4s avg %8.2f us' % (r['Name'][:34], r['Calls'], float(r['AverageNs'])/1e3))
PY
find $OUT/prof -name "*kernel_trace.csv" -size +4M -delete
