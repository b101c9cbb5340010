# two-tier listed items: parity, then A/B of the top tier's factor (0 = one tier)
set -u
OUT=gpurun_out/r4v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_tile_reuse.py tests/test_gpu_multirank.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" $OUT/tests.log | head -20; exit $rc; }
run() {  # tag env...
  local T=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$T.json 2> $OUT/bench_$T.err || { tail -3 $OUT/bench_$T.err; return 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$T.json'))
print('$T ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
}
for i in 1 2 3; do
  run x0_$i BSA_PF_HEAVY_X=0 || exit 1
  run x2_$i BSA_PF_HEAVY_X=2 || exit 1
  run x3_$i BSA_PF_HEAVY_X=3 || exit 1
  run x4_$i BSA_PF_HEAVY_X=4 || exit 1
  run x3p1n2_$i BSA_PF_HEAVY_X=3 BSA_PF_PIECES=1 BSA_PF_PIECES_NEAR=2 || exit 1
done
