# One PMC counter set for several library builds (A/B of memory behaviour).
# usage: LIBS="a:libX.so b:libY.so" SET="TCC_HIT_sum,TCC_MISS_sum" bash tools/pmc_ab.sh
set -u
mkdir -p gpurun_out/pmcab
export TMPDIR=/tmp
for cfg in $LIBS; do
  name=${cfg%%:*}; lib=${cfg#*:}
  BSACCEL_LIB=$PWD/bluesky_amd/$lib timeout -k 10 120 rocprofv3 --pmc ${SET//,/ } --kernel-trace --output-format csv \
      -d gpurun_out/pmcab/$name -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-variants \
      > gpurun_out/pmcab/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - gpurun_out/pmcab/$name <<'PY'
import csv, collections, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0])))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if 'k_prefilter' in r['Kernel_Name']:
        acc[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
print('  ' + '  '.join('%s %.4g' % (c, sum(d.values()) / len(d)) for c, d in sorted(acc.items())))
PY
done
