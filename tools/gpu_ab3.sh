# round 3: K0e item lists -- A/B of the split thresholds against the legacy
# item numbering (headline bench + per-rank probe).  PYTEST=1 runs a parity
# subset first.
set -u
mkdir -p gpurun_out/ab3
T="timeout -k 10"
if [ "${PYTEST:-0}" = 1 ]; then
  $T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
     tests/test_gpu_detect.py tests/test_gpu_fullsize.py::test_noprune_row_sweep_100k_bitwise \
     tests/test_gpu_multirank.py::test_halo_probe_shares_equal_full_detect tests/test_gpu_sim.py \
     tests/test_gpu_reuse.py > gpurun_out/ab3/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab3/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
REPS=${REPS:-2} CONFIGS=${CONFIGS:-"legacy:libbsaccel.so:BSA_PF_LEGACY=1 s12:libbsaccel.so:BSA_PF_SPLIT=12x24 s8:libbsaccel.so:BSA_PF_SPLIT=8x16 s16:libbsaccel.so:BSA_PF_SPLIT=16x32 s6:libbsaccel.so:BSA_PF_SPLIT=6x12 nosplit:libbsaccel.so:BSA_PF_SPLIT=64x64"} bash tools/ab_pf.sh || exit 1
for cfg in ${PROBES:-"legacy:BSA_PF_LEGACY=1" "list:BSA_PF_SPLIT=12x24"}; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs $T 300 python tools/rowslice_probe.py > gpurun_out/ab3/rs_$name.log 2>&1 || { tail -3 gpurun_out/ab3/rs_$name.log; exit 1; }
  echo "== probe $name"; cut -c1-200 gpurun_out/ab3/rs_$name.log
done
