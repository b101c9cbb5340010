# Prefilter diagnostics (diagnostic builds: `make -C bluesky_amd/csrc stamps trace`):
# phase stamps of three host detects at box100k (tools/stamps.py), then the
# per-item timeline (tools/pf_trace.py) of each TRACES entry ("WORKLOAD RANKS").
set -u
OUT=gpurun_out/${TAG:-diag}
mkdir -p $OUT
if [ "${STAMPS:-1}" = 1 ]; then
  BSACCEL_AB=1 BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_stamps.so timeout -k 10 120 python tools/stamps.py > $OUT/stamps.log 2>&1
  rc=$?; cat $OUT/stamps.log; [ $rc -eq 0 ] || exit $rc
fi
export BSACCEL_AB=1 BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_trace.so
echo "${TRACES:-box100k 1}" | tr ";" "\n" | while read wl r rk; do
  [ -n "$wl" ] || continue
  BSA_PF_TRACE_FILE=$OUT/tr.bin timeout -k 10 120 python tools/pf_trace.py run $wl $r ${rk:-0} || exit 1
  python tools/pf_trace.py show $OUT/tr.bin > $OUT/show_${wl}_$r.txt; echo "== trace $wl R=$r"; head -24 $OUT/show_${wl}_$r.txt
  rm -f $OUT/tr.bin
done
