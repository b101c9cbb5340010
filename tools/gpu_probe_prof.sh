# Kernel stats of one rank's share of the sharded step (tools/probe_step.py,
# global1m rank RANK of R, collectives excluded) and of the box100k bench, one
# summary line per kernel.  PYTEST="..." runs those GPU tests first.
set -u
OUT=gpurun_out/${TAG:-pprof}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "${PYTEST:-}" ]; then
  timeout -k 10 1000 python -u -m pytest $PYTEST -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
summ() {
  python3 - "$(find $1 -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:14]:
    print('  %-58s calls %6s avg %8.2f us' % (r['Name'][:58], r['Calls'], float(r['AverageNs']) / 1e3))
PY
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/probe -o run --output-format csv -- \
    python3 tools/probe_step.py global1m ${R:-8} 40 ${RANK:-4} > $OUT/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep "ms per step" $OUT/probe.log; [ $rc -eq 0 ] || exit $rc
summ $OUT/probe
find $OUT/probe -name "*kernel_trace.csv" -size +4M -delete
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run --output-format csv -- \
      python3 bench.py --steps 60 --warmup 10 --no-cpu --no-variants > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc $(python3 -c "import json; print(json.load(open('$OUT/bench.json'))['ms_per_step'])")"
  [ $rc -eq 0 ] || exit $rc
  summ $OUT/bench
  find $OUT/bench -name "*kernel_trace.csv" -size +4M -delete
fi
