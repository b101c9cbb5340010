# K0e diagnostics: kernel time of k_items under grid / mode knobs (rocprofv3 kernel trace of short benches)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/k0e
for cfg in "g2048 BSA_K0E_GRID=2048" "g512 BSA_K0E_GRID=512" "g256 BSA_K0E_GRID=256" "g4096 BSA_K0E_GRID=4096" "m1 BSA_K0E_MODE=1" "m2 BSA_K0E_MODE=2"; do
  set -- $cfg
  env $2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/k0e/$1 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-variants > gpurun_out/k0e/$1.log 2>&1 || { tail -5 gpurun_out/k0e/$1.log; exit 1; }
  python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/k0e/$1/run_kernel_stats.csv')))
print('$1', ' '.join('%s=%.1f' % (x['Name'].split('(')[0].split('::')[-1][:14], float(x['AverageNs'])/1e3) for x in r if any(k in x['Name'] for k in ('k_items','k_prefilter','k_tilepairs'))))"
done
