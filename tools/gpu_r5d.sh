# round 5: fused K1b A/B (heavy listing in k_rowblk's extra blocks)
set -u
OUT=gpurun_out/r5d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_detect.py tests/test_gpu_sim.py tests/test_gpu_tile_reuse.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="fused:libbsaccel.so sep:libbsaccel.so:BSA_FUSE_EXACT=0" REPS=3 TAG=r5d/ab bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > $OUT/prof.log 2>&1 || exit 1
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r5d/stats/**/*kernel_stats.csv', recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:6]:
    print('%-50s calls %5s avg %8.2f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
