# Kernel-trace stats of the headline bench (no CPU / variants); prints the
# per-kernel average durations.  LIB selects the library (default the in-tree one).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pq}
LIB=${LIB:-libbsaccel.so}
BSACCEL_LIB=$PWD/bluesky_amd/$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$TAG.log; exit $rc; }
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:16]:
    print('%-60s calls %5s avg %8.2f us  tot %8.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e3))
PY
