# Quick GPU check after a kernel change: detect parity (incl. the full-size
# NOPRUNE sweeps), the resident step, then the headline bench line.
set -u
mkdir -p gpurun_out
TAG=${TAG:-quick}
timeout -k 10 600 python -u -m pytest tests/test_gpu_detect.py tests/test_gpu_fullsize.py tests/test_gpu_sim.py tests/test_gpu_reuse.py tests/test_gpu_trace.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_$TAG.err
python -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('ms/step %.4f' % d['ms_per_step'], 'kernels', {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()}, 'cand', d['n_candidates'])"
exit $rc
