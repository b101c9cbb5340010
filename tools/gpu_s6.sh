# multi-rank parity + probe + rank trace (gpu_s5), then the prefilter item timeline of the new build
set -u
bash tools/gpu_s5.sh || exit 1
OUT=gpurun_out/s6
mkdir -p $OUT
BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_trace.so BSA_PF_TRACE_FILE=$OUT/tr.bin timeout -k 10 120 python tools/pf_trace.py run box100k 1 || exit 1
python tools/pf_trace.py show $OUT/tr.bin > $OUT/show_box100k_1.txt; head -16 $OUT/show_box100k_1.txt
python - <<PY
import numpy as np
raw=np.fromfile('$OUT/tr.bin',dtype=np.uint64)
np.save('$OUT/tr.npy', raw[:min(len(raw), 4000000)])
PY
rm -f $OUT/tr.bin
