# Per-rank probe (global1m) of the current build against a reference build.
set -u
mkdir -p gpurun_out/pab
for L in ${LIBS:-libbsaccel.so libbsaccel_ref.so}; do
  BSACCEL_LIB=$PWD/bluesky_amd/$L timeout -k 10 400 python tools/rowslice_probe.py ${WL:-global1m} > gpurun_out/pab/rs_$L.log 2>&1 || { tail -3 gpurun_out/pab/rs_$L.log; exit 1; }
  echo "== $L"; cut -c1-200 gpurun_out/pab/rs_$L.log
done
