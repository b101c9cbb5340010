# round 3: the new parity tests (sharded create/delete, every row of global1m,
# five 100k steps), then prefilter phase stamps and the item timeline
set -u
OUT=gpurun_out/diag
mkdir -p $OUT
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=0 -p no:cacheprovider \
   tests/test_gpu_multirank.py::test_sharded_create_delete_equal_world1 \
   tests/test_gpu_multirank.py::test_sharded_trace_super8del_equal_world1 \
   tests/test_gpu_fullsize.py > $OUT/pytest.log 2>&1
rc=$?; tail -30 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_stamps.so $T 120 python tools/stamps.py > $OUT/stamps.log 2>&1
rc=$?; cat $OUT/stamps.log; [ $rc -eq 0 ] || exit $rc
export BSACCEL_LIB=$PWD/bluesky_amd/libbsaccel_trace.so
BSA_PF_TRACE_FILE=$OUT/tr.bin $T 120 python tools/pf_trace.py run box100k 1 || exit 1
python tools/pf_trace.py show $OUT/tr.bin > $OUT/show_box100k_1.txt; head -30 $OUT/show_box100k_1.txt
rm -f $OUT/tr.bin
