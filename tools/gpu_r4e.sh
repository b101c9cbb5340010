# Round 4, pass e: parity incl. tile-pair list reuse, then TPR on/off on the bench, probe, stats.
set -u
OUT=gpurun_out/r4e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tile_reuse.py tests/test_gpu_fullsize.py::test_box100k_every_row_vs_oracle_fixture tests/test_gpu_fullsize.py::test_noprune_row_sweep_100k_bitwise tests/test_gpu_fullsize.py::test_resident_steps_100k_vs_oracle tests/test_gpu_asas_dropin.py tests/test_gpu_sim.py tests/test_gpu_trace.py tests/test_gpu_multirank.py tests/test_gpu_detect.py tests/test_gpu_mvp_kin.py tests/test_gpu_feed.py tests/test_gpu_reuse.py -m "gpu" -k "not 8ranks and not key_blocks" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for T in 1 0 1 0; do
  BSA_TPR=$T timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench_t$T.json 2> $OUT/bench_t$T.err || { tail -3 $OUT/bench_t$T.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_t$T.json'))
print('tpr $T ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
done
for G in 600 1200; do
  BSA_K1B_GRID=$G timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench_g$G.json 2> $OUT/bench_g$G.err || { tail -3 $OUT/bench_g$G.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_g$G.json'))
print('k1b grid $G ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > $OUT/prof_stats.log 2>&1
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/probe -o run --output-format csv -- \
    python tools/probe_rank.py global1m 8 2 20 > $OUT/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench_full.json 2> $OUT/bench_full.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('$OUT/bench_full.json')); print('asas_update', d.get('asas_update')); print('dropin', d.get('dropin_detect')); print('ms', d['ms_per_step'])"
