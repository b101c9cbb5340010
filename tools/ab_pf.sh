# A/B of prefilter variants on one box: each config runs the headline bench
# (no CPU, no variants) REPS times, interleaved; prints ms/step and stage times.
# usage: CONFIGS="name:LIB:ENV ..." bash tools/ab_pf.sh
set -u
mkdir -p gpurun_out
REPS=${REPS:-2}
for r in $(seq $REPS); do
  for cfg in $CONFIGS; do
    name=${cfg%%:*}; rest=${cfg#*:}; lib=${rest%%:*}; envs=${rest#*:}
    out=gpurun_out/ab_${name}_$r.json
    env BSACCEL_LIB=$PWD/bluesky_amd/$lib ${envs//,/ } timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $out 2> ${out%.json}.err
    rc=$?
    [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 ${out%.json}.err; exit $rc; }
    python -c "
import json; d=json.load(open('$out')); k=d['kernels_ms_rank0']
print('%-14s ms/step %.4f  k0 %.4f pf %.4f ex %.4f k2 %.4f cand %d' % ('$name', d['ms_per_step'], k['k0_prep'], k['prefilter'], k['exact'], k['k2_sort'], d['n_candidates']))"
  done
done
