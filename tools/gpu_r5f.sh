# round 5: merged halo plan + lists launch -- multirank parity, per-rank step probe
set -u
OUT=gpurun_out/r5g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_sim.py tests/test_gpu_detect.py tests/test_gpu_asas_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_step.py global1m 8 40 > $OUT/probe_step.log 2>&1 || { tail -3 $OUT/probe_step.log; exit 1; }
tail -1 $OUT/probe_step.log
timeout -k 10 400 python -u tools/rowslice_probe.py global1m box100k > $OUT/rowslice_probe.log 2>&1 || { tail -3 $OUT/rowslice_probe.log; exit 1; }
grep "R=8" $OUT/rowslice_probe.log | cut -c1-250
CONFIGS="base:libbsaccel.so r448:libbsaccel_r448.so r384:libbsaccel_r384.so" REPS=3 TAG=r5g/ab bash tools/gpu_ab.sh || exit 1
