# round 3: new drop-in + halo tests first, then the whole GPU suite, then the row-slice probe
set -u
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_asas_dropin.py \
   tests/test_gpu_multirank.py > gpurun_out/pytest_s2a.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_s2a.log; [ $rc -eq 0 ] || exit $rc
$T 600 python -u tools/rowslice_probe.py > gpurun_out/rowslice_s2.log 2>&1
rc=$?; cat gpurun_out/rowslice_s2.log | tail -12; [ $rc -eq 0 ] || exit $rc
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_s2b.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_s2b.log; exit $rc
