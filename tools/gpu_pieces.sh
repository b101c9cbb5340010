# A/B of the prefilter's item pieces (BSA_PF_PIECES = 1 / 2 / 4): headline
# bench and the per-rank probe for each setting.
set -u
OUT=gpurun_out/pieces
mkdir -p $OUT
for P in ${PIECES:-1 2 4}; do
  export BSA_PF_PIECES=$P
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench_$P.json 2> $OUT/bench_$P.err || { tail -3 $OUT/bench_$P.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$P.json'))
print('pieces $P ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
  timeout -k 10 300 python tools/rowslice_probe.py > $OUT/rs_$P.log 2>&1 || { tail -3 $OUT/rs_$P.log; exit 1; }
  python -c "
import json
for l in open('$OUT/rs_$P.log'):
    a, r, j = l.split(' ', 2); d = json.loads(j); print('   ', a, r, d['ms'])"
done
