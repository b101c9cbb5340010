# A/B of library builds on the per-rank probe (box100k rows of R ranks)
# usage: bash tools/gpu_probe_ab.sh LIB_A LIB_B ...
set -u
OUT=gpurun_out/pab
mkdir -p $OUT
for L in "$@"; do
  BSACCEL_LIB=$PWD/bluesky_amd/$L timeout -k 10 200 python -u tools/rowslice_probe.py box100k > $OUT/rs_$L.log 2>&1 || { tail -3 $OUT/rs_$L.log; exit 1; }
  echo "== $L"; cut -c1-140 $OUT/rs_$L.log
done
