# A/B of library variants on the headline bench + the per-rank probe (box100k R=1/8, 1M R=1/8).
set -u
OUT=gpurun_out/ab
mkdir -p $OUT
for L in ${LIBS:-libbsaccel.so}; do
  export BSACCEL_LIB=$PWD/bluesky_amd/$L
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench_$L.json 2> $OUT/bench_$L.err || { tail -3 $OUT/bench_$L.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$L.json'))
print('$L ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
  timeout -k 10 300 python tools/rowslice_probe.py > $OUT/rs_$L.log 2>&1 || { tail -3 $OUT/rs_$L.log; exit 1; }
  grep -E "R=1 |R=8 " $OUT/rs_$L.log | python -c "
import sys, json
for l in sys.stdin:
    a, r, j = l.split(' ', 2); d = json.loads(j); print('   ', a, r, d['ms'])"
done
