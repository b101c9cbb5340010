# Kernel-stats A/B: rocprofv3 --kernel-trace --stats of the box100k bench for
# each CONFIGS entry ("name:LIB[:ENV=V,...]"), one summary line per kernel.
#   CONFIGS="head:libbsaccel_head.so new:libbsaccel.so:BSA_HK=0" bash tools/gpu_kstats.sh
set -u
OUT=gpurun_out/${TAG:-kstats}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in ${CONFIGS:-base:libbsaccel.so}; do
  name=${cfg%%:*}; rest=${cfg#*:}; lib=${rest%%:*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*:}
  export BSACCEL_AB=1 BSACCEL_LIB=$PWD/bluesky_amd/$lib
  for e in ${envs//,/ }; do export "$e"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run --output-format csv -- \
      python3 bench.py --steps ${STEPS:-60} --warmup 10 --no-cpu --no-variants ${BENCH_ARGS:-} > $OUT/$name.json 2> $OUT/$name.err
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 $OUT/$name.err; exit $rc; }
  for e in ${envs//,/ }; do unset "${e%%=*}"; done
  f=$(find $OUT/$name -name '*kernel_stats.csv' | head -1)
  echo "== $name $(python3 -c "import json; print(json.load(open('$OUT/$name.json'))['ms_per_step'])")"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:12]:
    print('  %-60s calls %6s avg %8.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
