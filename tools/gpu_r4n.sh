# Round 4: per-rank share of a CD step (plan + list reuse): rowslice_probe
# (stage times of every rank's detect, slowest rank) and the kernel trace of
# rank 2 of 8 at global1m with reuse off / on.
set -u
OUT=gpurun_out/r4n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/rowslice_probe.py box100k global1m > $OUT/rowslice_probe.log 2>&1; rc=$?
cat $OUT/rowslice_probe.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for A in 0 1; do
  BSA_TPR=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/probe_tpr$A -o run --output-format csv -- \
      python tools/probe_rank.py global1m 8 2 20 > $OUT/probe_tpr$A.log 2>&1
  rc=$?; echo "probe tpr=$A rc=$rc"; grep "per detect" $OUT/probe_tpr$A.log; [ $rc -eq 0 ] || exit $rc
  python - <<PY
import csv, glob
f = glob.glob('$OUT/probe_tpr$A/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print('tpr=$A %-34s calls %4s avg %8.2f us' % (r['Name'][:34], r['Calls'], float(r['AverageNs'])/1e3))
PY
  find $OUT/probe_tpr$A -name "*kernel_trace.csv" -size +4M -delete
done
