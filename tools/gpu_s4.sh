# round 3 session: parity subset + A/B (ref = HEAD build, new = working tree),
# then kernel traces of the headline bench and of one rank's share at R = 8
set -u
export TMPDIR=/tmp
PYTEST=1 CONFIGS="ref:libbsaccel_ref.so:X=1 new:libbsaccel.so:X=1 k4b64:libbsaccel.so:BSA_K4_BLOCK=64 k4b128:libbsaccel.so:BSA_K4_BLOCK=128" PROBES="new:X=1" bash tools/gpu_ab3.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab3/stats -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > gpurun_out/ab3/stats.log 2>&1 || exit 1
for wl in "global1m 8 4" "box100k 8 0"; do
  set -- $wl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab3/rank_$1 -o run --output-format csv -- python tools/probe_rank.py $1 $2 $3 20 > gpurun_out/ab3/rank_$1.log 2>&1 || { tail -5 gpurun_out/ab3/rank_$1.log; exit 1; }
  grep "per detect" gpurun_out/ab3/rank_$1.log
done
