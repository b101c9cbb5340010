# GPU-box check: parity tests, then (if no crash) the bench and a kernel-trace profile.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROF:-1}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_$TAG -name '*stats*' | head
  [ $rc -eq 0 ] || exit $rc
fi
