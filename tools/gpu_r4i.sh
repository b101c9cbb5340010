# Round 4: K0d fused into the prefilter (builds only) -- parity, then A/B
# against the separate launch (BSA_K0D_FUSE=0) and K1b grid sizes.
set -u
OUT=gpurun_out/r4i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread \
    tests/test_gpu_tile_reuse.py tests/test_gpu_multirank.py tests/test_gpu_sim.py tests/test_gpu_detect.py \
    > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for V in "BSA_K0D_FUSE=1" "BSA_K0D_FUSE=0" "BSA_K1B_GRID=768" "BSA_K1B_GRID=1024" "BSA_K0D_FUSE=1" "BSA_K0D_FUSE=0" "BSA_K1B_GRID=768" "BSA_K1B_GRID=1024"; do
  env $V timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/bench_$V.json 2> $OUT/bench_$V.err || { tail -3 $OUT/bench_$V.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$V.json'))
print('$V ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()}, d.get('tile_reuse_rank0'))"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python bench.py --steps 40 --warmup 3 --no-cpu --no-variants > $OUT/prof.log 2>&1; echo "prof rc=$?"
