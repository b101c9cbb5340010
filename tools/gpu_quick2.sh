# Parity (detect, full-size sweeps, sim, multi-rank, reuse, traces), the
# headline bench and the per-rank probe -- one GPU call after a kernel change.
set -u
TAG=${TAG:-q2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_detect.py tests/test_gpu_fullsize.py tests/test_gpu_sim.py tests/test_gpu_multirank.py tests/test_gpu_reuse.py tests/test_gpu_trace.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print('ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
timeout -k 10 300 python tools/rowslice_probe.py > $OUT/rowslice.log 2>&1
rc=$?; python -c "
import json
for l in open('$OUT/rowslice.log'):
    a, r, j = l.split(' ', 2); d = json.loads(j); print('   ', a, r, d['ms'])"
exit $rc
