# Round 4, pass c: the new fixture test + host-path changes (parity), the K2
# block-size A/B, the per-rank kernel trace at global1m R=8, PMC of the build,
# and one full bench line (variants incl. asas_update).
set -u
OUT=gpurun_out/r4c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py::test_box100k_every_row_vs_oracle_fixture tests/test_gpu_asas_dropin.py tests/test_gpu_sim.py tests/test_gpu_trace.py tests/test_gpu_multirank.py tests/test_gpu_detect.py -m "gpu" -k "not 8ranks and not key_blocks" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for L in libbsaccel.so libbsaccel_rr256.so libbsaccel_rr128.so libbsaccel.so libbsaccel_rr256.so libbsaccel_rr128.so; do
  BSACCEL_LIB=$PWD/bluesky_amd/$L timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-variants > $OUT/bench_$L.json 2> $OUT/bench_$L.err || { tail -3 $OUT/bench_$L.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$L.json'))
print('$L ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
done
for A in 0 1; do
  BSA_TP_HALO_ALL=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/probe_tp$A -o run --output-format csv -- \
      python tools/probe_rank.py global1m 8 2 20 > $OUT/probe_tp$A.log 2>&1
  rc=$?; echo "probe tp_all=$A rc=$rc"; tail -1 $OUT/probe_tp$A.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > $OUT/prof_stats.log 2>&1
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/pmc_p$i -o run -- \
      python bench.py --steps 3 --warmup 1 --no-cpu --no-variants > $OUT/pmc_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench_full.json 2> $OUT/bench_full.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('$OUT/bench_full.json')); print('asas_update', d.get('asas_update')); print('reuse', d['variants']['candidate_reuse']['ms_per_step'])"
