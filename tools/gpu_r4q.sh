# K2 payloads by bucket slot (K1b writes them beside the bucket entry; K2
# loads both at once): parity, then A/B against the base build
set -u
OUT=gpurun_out/r4q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_detect.py tests/test_gpu_sim.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py \
    tests/test_gpu_asas_dropin.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab2.sh libbsaccel_base.so libbsaccel.so 3
