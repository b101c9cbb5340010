# K1b's listing pass on the lanes after the candidates: parity, then A/B vs base
set -u
OUT=gpurun_out/r4x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_tile_reuse.py tests/test_gpu_multirank.py tests/test_gpu_detect.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" $OUT/tests.log | head -20; exit $rc; }
bash tools/gpu_ab2.sh libbsaccel_base.so libbsaccel.so 3
