set -u
OUT=gpurun_out/pf2
mkdir -p $OUT
export BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_trace.so
for a in "box100k 1" "box100k 8"; do
  set -- $a
  BSA_PF_TRACE_FILE=$OUT/tr.bin timeout -k 10 120 python tools/pf_trace.py run $1 $2 || exit 1
  echo "== trace $1 R=$2"; python tools/pf_trace.py show $OUT/tr.bin > $OUT/show_$1_$2.txt; head -24 $OUT/show_$1_$2.txt
  python - <<PY
import numpy as np
raw=np.fromfile('$OUT/tr.bin',dtype=np.uint64)
np.save('$OUT/tr_$1_$2.npy', raw[:min(len(raw), 4000000)])
PY
  rm -f $OUT/tr.bin
done
