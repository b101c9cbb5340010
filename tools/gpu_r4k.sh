# K0d fused vs separate: kernel stats of the bench under rocprofv3 (both)
set -u
OUT=gpurun_out/r4k
mkdir -p $OUT
export TMPDIR=/tmp
for F in 1 0; do
  BSA_K0D_FUSE=$F timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/prof_f$F -o run --output-format csv -- \
      python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/prof_f$F.log 2>&1; rc=$?; echo "prof fuse=$F rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - <<PY
import csv, glob
f = glob.glob('$OUT/prof_f$F/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print('fuse=$F %-34s calls %4s avg %8.2f us total %9.1f us' % (r['Name'][:34], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e3))
PY
  find $OUT/prof_f$F -name "*kernel_trace.csv" -size +4M -delete
done
