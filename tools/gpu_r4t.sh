# longest items first (same pieces): parity, then A/B (BSA_PF_HEAVY=0 / 1, thresholds)
set -u
OUT=gpurun_out/r4t
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag env...
  local T=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$T.json 2> $OUT/bench_$T.err || { tail -3 $OUT/bench_$T.err; return 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$T.json'))
print('$T ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
}
for i in 1 2 3; do
  run h8_$i BSA_PF_HEAVY=1 BSA_PF_HEAVY_US=8 || exit 1
  run h12_$i BSA_PF_HEAVY=1 BSA_PF_HEAVY_US=12 || exit 1
  run h16_$i BSA_PF_HEAVY=1 BSA_PF_HEAVY_US=16 || exit 1
  run h20_$i BSA_PF_HEAVY=1 BSA_PF_HEAVY_US=20 || exit 1
done
