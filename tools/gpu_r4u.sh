# longest items first: parity (tile reuse incl. every / no item listed, sim, multirank, detect)
set -u
OUT=gpurun_out/r4u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_tile_reuse.py tests/test_gpu_sim.py tests/test_gpu_multirank.py tests/test_gpu_detect.py \
    tests/test_gpu_reuse.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" $OUT/tests.log | head -20; exit $rc; }
