# PMC counter passes on the bench (separate passes; kernel-trace only, no sys/runtime trace).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/${TAG}_p$i -o run -- \
      python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
