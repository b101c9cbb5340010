# round 3: halo regrowth + atmosphere tests, then the whole GPU suite, then the row-slice probe
set -u
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
   tests/test_gpu_multirank.py::test_halo_requests_and_regrowth_equal_world1 \
   tests/test_gpu_sim.py::test_resident_atmosphere_outputs > gpurun_out/pytest_s3a.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_s3a.log; [ $rc -eq 0 ] || exit $rc
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_s3b.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_s3b.log; [ $rc -eq 0 ] || exit $rc
$T 600 python -u tools/rowslice_probe.py > gpurun_out/rowslice_s3.log 2>&1
rc=$?; tail -12 gpurun_out/rowslice_s3.log; exit $rc
