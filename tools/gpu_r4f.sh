# Round 4, pass f: tile-pair list reuse budget A/B on the headline bench.
set -u
OUT=gpurun_out/r4f
mkdir -p $OUT
for V in 0:0 1:500 1:1000 1:2016 0:0 1:500 1:1000 1:2016; do
  T=${V%%:*}; S=${V##*:}
  BSA_TPR=$T BSA_TPR_SH=$S timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$T_$S.json 2> $OUT/bench.err || { tail -3 $OUT/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$T_$S.json'))
print('tpr $T sh $S ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()}, d['tile_reuse_rank0']['builds'], d['tile_reuse_rank0']['detects'])"
done
