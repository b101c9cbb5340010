# Prefilter work-split knobs A/B on the current build, then the per-rank probe.
set -u
mkdir -p gpurun_out/s9
REPS=${REPS:-2} CONFIGS=${CONFIGS:-"p2:libbsaccel.so: p1:libbsaccel.so:BSA_PF_PIECES=1 p4:libbsaccel.so:BSA_PF_PIECES=4 n1:libbsaccel.so:BSA_PF_PIECES_NEAR=1"} bash tools/ab_pf.sh || exit 1
timeout -k 10 400 python tools/rowslice_probe.py > gpurun_out/s9/rowslice_probe.log 2>&1 || { tail -3 gpurun_out/s9/rowslice_probe.log; exit 1; }
cut -c1-230 gpurun_out/s9/rowslice_probe.log
BSA_TP_SUPER=1 timeout -k 10 400 python tools/rowslice_probe.py global1m > gpurun_out/s9/rowslice_probe_super.log 2>&1 || { tail -3 gpurun_out/s9/rowslice_probe_super.log; exit 1; }
echo "== super K0d"; cut -c1-230 gpurun_out/s9/rowslice_probe_super.log
