# Dev iteration on the GPU box: parity tests, bench (no CPU leg), optional
# prefilter phase stamps from the diagnostic build.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/dev_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/dev_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/dev_bench.json 2> gpurun_out/dev_bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/dev_bench.json'))
print('ms/step %.4f  prefilter %.4f  exact %.4f  detect %.4f  cand %d  conf %d los %d' % (d['ms_per_step'], d['kernels_ms_rank0']['prefilter'], d['kernels_ms_rank0']['exact'], d['kernels_ms_rank0']['detect_total'], d['n_candidates'], d['n_conf'], d['n_los']))"
[ $rc -eq 0 ] || exit $rc
if [ -f bluesky_amd/libbsaccel_stamps.so ] && [ "${STAMPS:-1}" = 1 ]; then
  BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_stamps.so timeout -k 10 120 python tools/stamps.py > gpurun_out/dev_stamps.log 2>&1
  rc=$?; grep stamps gpurun_out/dev_stamps.log | tail -1; tail -1 gpurun_out/dev_stamps.log
  [ $rc -eq 0 ] || exit $rc
fi
