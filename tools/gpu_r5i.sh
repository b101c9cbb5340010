# round 5: in-kernel heavy listing -- parity, A/B against the previous library
set -u
OUT=gpurun_out/r5i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_tile_reuse.py tests/test_gpu_sim.py tests/test_gpu_detect.py tests/test_gpu_fullsize.py tests/test_gpu_trace.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="new:libbsaccel.so prev:libbsaccel_prev.so new24:libbsaccel.so:BSA_PF_HEAVY_US=24" REPS=4 TAG=r5i/ab bash tools/gpu_ab.sh || exit 1
