# Round 4, pass g: prefilter pieces A/B (far items split finer to shorten the sweep's tail).
set -u
OUT=gpurun_out/r4g
mkdir -p $OUT
for V in 2:2 4:2 4:1 8:2 2:2 4:2 4:1 8:2; do
  P=${V%%:*}; N=${V##*:}
  BSA_PF_PIECES=$P BSA_PF_PIECES_NEAR=$N timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_${P}_${N}.json 2> $OUT/bench.err || { tail -3 $OUT/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_${P}_${N}.json'))
print('pieces far $P near $N ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
done
