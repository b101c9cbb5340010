# Per-rank share of a sharded CD step on one GPU: the stage
# probe (tools/rowslice_probe.py) and a kernel-trace profile of one rank's
# detects (tools/probe_rank.py).  WL / R / RANK select the rank.
set -u
OUT=gpurun_out/${TAG:-probe}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/rowslice_probe.py ${PROBE_WL:-global1m box100k} > $OUT/rowslice_probe.log 2>&1
rc=$?; cut -c1-260 $OUT/rowslice_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rank -o run --output-format csv -- \
    python tools/probe_rank.py ${WL:-global1m} ${R:-8} ${RANK:-4} 20 > $OUT/probe_rank.log 2>&1
rc=$?; cat $OUT/probe_rank.log; [ $rc -eq 0 ] || exit $rc
python - $OUT/rank <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
tot = 0.0
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs'])):
    if int(r['Calls']) < 20:
        continue
    tot += float(r['AverageNs']) * int(r['Calls']) / 23
    print('%-60s calls %4s avg %7.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
print('kernels per detect (23 detects): %.1f us' % (tot / 1e3))
PY
find $OUT/rank -name "*kernel_trace.csv" -size +4M -delete
