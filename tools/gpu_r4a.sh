# Round 4, first GPU pass: parity (not slow), new vs round-3 library on the
# headline bench, the per-rank probe, a kernel-trace profile of the new build.
set -u
OUT=gpurun_out/r4a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for L in libbsaccel_r3.so libbsaccel.so libbsaccel_r3.so libbsaccel.so; do
  BSACCEL_LIB=$PWD/bluesky_amd/$L timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench_$L.json 2> $OUT/bench_$L.err || { tail -3 $OUT/bench_$L.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$L.json'))
print('$L ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()}, d['n_candidates'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > $OUT/prof_stats.log 2>&1
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/rowslice_probe.py > $OUT/rowslice_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat $OUT/rowslice_probe.log | cut -c1-400
