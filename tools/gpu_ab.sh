# A/B of library builds and environment knobs on the box100k headline bench,
# interleaved REPS times, plus (optionally) the per-rank probe.  Replaces the
# one-off round scripts: every earlier A/B is one CONFIGS line.
#
#   CONFIGS="name:LIB[:ENV=V,ENV=V] ..."   (default "base:libbsaccel.so")
#   REPS=3  STEPS=60  WARMUP=10  BENCH_ARGS="--workload global1m"
#   PROBE=1 (tools/rowslice_probe.py per config; PROBE_WL="box100k global1m")
#   STEP_PROBE="global1m 8 40 4" (tools/probe_step.py per config and rep: one rank's whole step)
#   PYTEST="tests/test_gpu_detect.py ..." (parity subset first, on the default library)
#
# e.g. CONFIGS="a:libbsaccel.so b:libbsaccel_x.so c:libbsaccel.so:BSA_PF_PIECES_NEAR=4" REPS=3 bash tools/gpu_ab.sh
set -u
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "${PYTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest $PYTEST -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq ${REPS:-3}); do
  for cfg in ${CONFIGS:-base:libbsaccel.so}; do
    name=${cfg%%:*}; rest=${cfg#*:}; lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*:}
    o=$OUT/b_${name}_$r
    env BSACCEL_AB=1 BSACCEL_LIB=$PWD/bluesky_amd/$lib ${envs//,/ } timeout -k 10 240 \
        python bench.py --steps ${STEPS:-60} --warmup ${WARMUP:-10} --no-cpu --no-variants ${BENCH_ARGS:-} > $o.json 2> $o.err
    rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 $o.err; exit $rc; }
    python -c "
import json; d=json.load(open('$o.json')); k=d['kernels_ms_rank0']
print('%-12s ms/step %.4f  k0 %.4f pf %.4f ex %.4f k2 %.4f  cand %d' % ('$name', d['ms_per_step'], k['k0_prep'], k['prefilter'], k['exact'], k['k2_sort'], d['n_candidates']))"
    if [ -n "${STEP_PROBE:-}" ]; then
      env BSACCEL_AB=1 BSACCEL_LIB=$PWD/bluesky_amd/$lib ${envs//,/ } timeout -k 10 240 \
          python -u tools/probe_step.py $STEP_PROBE > $o.step 2>&1 || { tail -3 $o.step; exit 1; }
      echo "$name step probe: $(grep 'ms per step' $o.step | tail -1)"
    fi
  done
done
if [ "${PROBE:-0}" = 1 ]; then
  for cfg in ${CONFIGS:-base:libbsaccel.so}; do
    name=${cfg%%:*}; rest=${cfg#*:}; lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*:}
    env BSACCEL_AB=1 BSACCEL_LIB=$PWD/bluesky_amd/$lib ${envs//,/ } timeout -k 10 400 \
        python -u tools/rowslice_probe.py ${PROBE_WL:-box100k global1m} > $OUT/rs_$name.log 2>&1 || { tail -3 $OUT/rs_$name.log; exit 1; }
    echo "== probe $name"; cut -c1-200 $OUT/rs_$name.log
  done
fi
