# bench with candidate-list reuse at several budgets (no CPU leg)
set -u
mkdir -p gpurun_out
for cfg in "" "800 60" "1500 150" "2500 150" "1500 300"; do
  if [ -z "$cfg" ]; then arg=""; else arg="--reuse $cfg"; fi
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu $arg > gpurun_out/abr.json 2> gpurun_out/abr.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/abr.err; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/abr.json')); k=d['kernels_ms_rank0']
print('%-12s ms/step %.4f  prefilter %.4f exact %.4f k2 %.4f k0 %.4f detect %.4f cand %d reuse %s' % (sys.argv[1], d['ms_per_step'], k['prefilter'], k['exact'], k['k2_sort'], k['k0_prep'], k['detect_total'], d['n_candidates'], d['reuse']))" "${cfg:-off}"
done
