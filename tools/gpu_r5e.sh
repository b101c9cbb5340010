# round 5: prefilter stamps (fused) + item trace, and the kernel trace of one rank's whole step at global1m R=8
set -u
OUT=gpurun_out/r5e
mkdir -p $OUT
export TMPDIR=/tmp
TAG=r5e STAMPS=1 TRACES="box100k 1" bash tools/gpu_diag.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/step -o run --output-format csv -- \
    python tools/probe_step.py global1m 8 30 4 > $OUT/probe_step4.log 2>&1
rc=$?; tail -2 $OUT/probe_step4.log; [ $rc -eq 0 ] || exit $rc
python - $OUT/step <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:16]:
    print('%-60s calls %4s avg %7.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
python tools/trace_gaps.py $(find $OUT/step -name "*kernel_trace.csv" | head -1) > $OUT/step_gaps.txt 2>&1; tail -5 $OUT/step_gaps.txt
find $OUT/step -name "*kernel_trace.csv" -size +4M -delete
