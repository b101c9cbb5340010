# A/B/... of several library builds on the box100k bench (alternating, 60 steps each)
# usage: bash tools/gpu_abn.sh REPS LIB_A LIB_B [LIB_C ...]
set -u
OUT=gpurun_out/abn
mkdir -p $OUT
export TMPDIR=/tmp
N=$1; shift
for i in $(seq 1 $N); do
  for L in "$@"; do
    BSACCEL_LIB=$PWD/bluesky_amd/$L timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu --no-variants > $OUT/b_${L}_$i.json 2> $OUT/b_${L}_$i.err || { tail -3 $OUT/b_${L}_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/b_${L}_$i.json'))
print('$L ms/step %.4f' % d['ms_per_step'], {k: round(v, 4) if isinstance(v, float) else v for k, v in d['kernels_ms_rank0'].items()})"
  done
done
