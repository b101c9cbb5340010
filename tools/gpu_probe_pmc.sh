# PMC passes over one rank's step of the sharded global1m step (probe_step.py,
# rank 4 of 8): per-kernel memory-side bytes and instruction mix.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05q}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python tools/probe_step.py global1m 8 30 4 50 > $OUT/stats.log 2>&1 || exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python tools/probe_step.py global1m 8 10 4 0 > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_roofline.py $OUT/pmc_probe.json $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 > /dev/null
find $OUT -name "*kernel_trace.csv" -size +4M -delete
python - <<'PY'
import json, os
d = json.load(open(os.environ.get('OUT', 'gpurun_out/r05q') + '/pmc_probe.json'))
for k, v in d.items():
    if k.startswith('_'): continue
    print(k[:40], {a: round(b / 1e6, 3) if isinstance(b, float) and b > 1e4 else b for a, b in v.items()})
PY
