# prefilter pieces with the longest-items listing on: near pieces 2 (default) / 1 / 4
set -u
OUT=gpurun_out/r4y
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag env...
  local T=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 60 --warmup 10 --no-cpu --no-variants > $OUT/bench_$T.json 2> $OUT/bench_$T.err || { tail -3 $OUT/bench_$T.err; return 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$T.json'))
print('$T ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
}
for i in 1 2 3; do
  run pn2_$i BSA_PF_PIECES_NEAR=2 || exit 1
  run pn1_$i BSA_PF_PIECES_NEAR=1 || exit 1
  run pn4_$i BSA_PF_PIECES_NEAR=4 || exit 1
done
