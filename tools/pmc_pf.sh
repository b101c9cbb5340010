# Prefilter diagnostics: available counters, phase stamps (diagnostic build),
# then --pmc passes of the headline bench (one counter set per run).
set -u
mkdir -p gpurun_out/pmcpf
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/pmcpf/avail.txt 2>&1
BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_stamps.so timeout -k 10 120 python tools/stamps.py > gpurun_out/pmcpf/stamps.txt 2>&1
rc=$?; echo "stamps rc=$rc"; tail -2 gpurun_out/pmcpf/stamps.txt; [ $rc -eq 0 ] || exit $rc
i=0
for set in ${SETS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc ${set//,/ } --kernel-trace --output-format csv -d gpurun_out/pmcpf/p$i -o run -- \
      python bench.py --steps 3 --warmup 1 --no-cpu --no-variants > gpurun_out/pmcpf/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
