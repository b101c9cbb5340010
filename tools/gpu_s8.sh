# K4' prepares the next detect's records: the GPU suite, A/B (ref = HEAD~, prep on / off), kernel stats
set -u
export TMPDIR=/tmp
OUT=gpurun_out/s8
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=2 CONFIGS="ref:libbsaccel_ref.so:X=1 prep:libbsaccel.so:X=1 noprep:libbsaccel.so:BSA_SIM_PREP=0" PROBES="x:X=1" bash tools/gpu_ab3.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > $OUT/stats.log 2>&1 || exit 1
