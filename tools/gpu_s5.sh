# halo launch reduction: multi-rank parity, then A/B (ref = HEAD) + one rank's kernel trace
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s5
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
   tests/test_gpu_multirank.py > gpurun_out/s5/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/s5/pytest.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="ref:libbsaccel_ref.so:X=1 new:libbsaccel.so:X=1" PROBES="new:X=1" bash tools/gpu_ab3.sh || exit 1
for wl in "global1m 8 4" "box100k 8 0"; do
  set -- $wl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s5/rank_$1 -o run --output-format csv -- python tools/probe_rank.py $1 $2 $3 20 > gpurun_out/s5/rank_$1.log 2>&1 || { tail -5 gpurun_out/s5/rank_$1.log; exit 1; }
  grep "per detect" gpurun_out/s5/rank_$1.log
done
