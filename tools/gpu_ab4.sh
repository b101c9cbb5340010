# Parity subset on the current build, then an A/B of CONFIGS against the
# reference build and a kernel-trace --stats profile of the current build.
set -u
OUT=gpurun_out/${TAG:-ab4}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${PYTEST:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
     ${TESTS:-tests/test_gpu_detect.py tests/test_gpu_sim.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py tests/test_gpu_trace.py} \
     > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
REPS=${REPS:-2} CONFIGS=${CONFIGS:-"new:libbsaccel.so: ref:libbsaccel_ref.so:"} bash tools/ab_pf.sh || exit 1
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
      python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > $OUT/prof_stats.log 2>&1
  rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - <<PY
import csv, glob
f = glob.glob('$OUT/stats/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print('%-40s %6s %10.1f' % (r['Name'][:40], r['Calls'], float(r['AverageNs']) / 1e3))
PY
fi
