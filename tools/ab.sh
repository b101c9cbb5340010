# A/B timing of library builds on the GPU box: bench (no CPU leg) per .so.
# usage: bash tools/ab.sh bluesky_amd/libbsaccel.so bluesky_amd/libbsaccel_x.so ...
set -u
mkdir -p gpurun_out
for lib in "$@"; do
  for rep in 1 2; do
    BSACCEL_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?
    [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 gpurun_out/ab.err; exit $rc; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab.json')); k=d['kernels_ms_rank0']
print('%-40s ms/step %.4f  prefilter %.4f exact %.4f k2 %.4f k0 %.4f detect %.4f' % (sys.argv[1], d['ms_per_step'], k['prefilter'], k['exact'], k['k2_sort'], k['k0_prep'], k['detect_total']))" "$lib"
  done
done
