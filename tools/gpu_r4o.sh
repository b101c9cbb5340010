# prefilter with the next unit's dequeue + item prefetched: detect parity
# (all-rows pruned == NOPRUNE, fixtures), then A/B against the base build
set -u
OUT=gpurun_out/r4o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_detect.py tests/test_gpu_tile_reuse.py tests/test_gpu_fullsize.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh libbsaccel_base.so libbsaccel.so 3
