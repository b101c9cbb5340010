# GPU check of the resident path: all GPU tests, the headline bench line, and
# the summed per-kernel work of 1 / 2 / 4 / 8 in-process ranks (rocprofv3 stats).
set -u
TAG=${TAG:-home}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print('ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
for W in ${WORLDS:-1 2 4 8}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/grp_${WL:-box100k}_$W -o run --output-format csv -- \
      python tools/group_probe.py ${WL:-box100k} $W 10 > $OUT/grp_${WL:-box100k}_$W.log 2>&1
  rc=$?; echo "group $W rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/grp_${WL:-box100k}_$W.log; exit $rc; }
done
