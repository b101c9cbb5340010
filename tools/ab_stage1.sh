# GPU A/B of the prefilter's stage-1 geometry: look-ahead midpoints (default)
# vs t = 0 positions (BSA_STAGE1_T0=1), after the parity tests.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ab1_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/ab1_pytest.log
[ $rc -eq 0 ] || exit $rc
for mode in mid t0; do
  if [ $mode = t0 ]; then export BSA_STAGE1_T0=1; else unset BSA_STAGE1_T0; fi
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab1_$mode.json 2> gpurun_out/ab1_$mode.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/ab1_$mode.err; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab1_$mode.json')); k=d['kernels_ms_rank0']
print('%-4s ms/step %.4f  prefilter %.4f exact %.4f k2 %.4f k0 %.4f detect %.4f  tiles %.0f tests %.3g cand %d conf %d los %d' % ('$mode', d['ms_per_step'], k['prefilter'], k['exact'], k['k2_sort'], k['k0_prep'], k['detect_total'], d['tile_pairs_rank0'], d['prefilter_pair_tests_rank0'], d['n_candidates'], d['n_conf'], d['n_los']))"
done
