set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/stats -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu --no-variants > gpurun_out/ev/prof.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ev/bench.json 2> gpurun_out/ev/bench.err || exit $?
cat gpurun_out/ev/bench.json | cut -c1-300
