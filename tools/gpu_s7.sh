# refine diet + halo launch cuts: exactness at full size, multi-rank parity, A/B vs HEAD, probe, item timeline
set -u
export TMPDIR=/tmp
OUT=gpurun_out/s7
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
   tests/test_gpu_detect.py tests/test_gpu_fullsize.py tests/test_gpu_reuse.py tests/test_gpu_multirank.py \
   tests/test_gpu_sim.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="ref:libbsaccel_ref.so:X=1 new:libbsaccel.so:X=1" PROBES="new:X=1" bash tools/gpu_ab3.sh || exit 1
BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_trace.so BSA_PF_TRACE_FILE=$OUT/tr.bin timeout -k 10 120 python tools/pf_trace.py run box100k 1 || exit 1
python tools/pf_trace.py show $OUT/tr.bin > $OUT/show_box100k_1.txt; head -8 $OUT/show_box100k_1.txt
python - <<PY
import numpy as np
raw=np.fromfile('$OUT/tr.bin',dtype=np.uint64)
np.save('$OUT/tr.npy', raw[:min(len(raw), 4000000)])
PY
rm -f $OUT/tr.bin
