#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric on MI355X: CD pair-evals/s at 100k aircraft.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE
JSON line on rank 0.  A step = one StateBased detect pass over the synthetic
100k-aircraft density-matched box (BASELINE.json configs[3]),
inputs already resident in HBM: prep + prefilter + exact fp64 evaluation +
canonical sort, all N^2 pairs (diagonal included in the count).
``value`` = N^2 * steps / time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from bluesky_amd import _lib, synth  # noqa: E402

FP64_PEAK_TFLOPS = 78.6      # MI355X fp64 vector (spec; FMA = 2)
FP32_PEAK_TFLOPS = 157.3     # MI355X fp32 vector (MI355X_MICROARCH.md)
OPS_PER_PAIR = 110           # algorithmic fp64 ops per pair-eval
PF_FLOPS_PER_PAIR = 16       # prefilter: 3 sub, 1 mul + 2 fma (x2), add, mul, sub, add, 2 cmp


def cpu_baseline(t, rows_sample, seed=0):
    """Oracle (numpy restatement, 1 process) on a uniform row sample."""
    from oracle import statebased as ocd
    n = t.ntraf
    rows = np.linspace(0, n - 1, rows_sample).astype(np.int64)
    t0 = time.perf_counter()
    ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, rows=rows, budget_bytes=1 << 30)
    dt = time.perf_counter() - t0
    pairs = rows_sample * n
    return dict(value=pairs / dt, unit='pair-evals/s', cores=1, kind='port',
                sample='%d uniformly spaced ownship rows x %d columns (%.1f s), numpy %s, '
                       'single process, OPENBLAS_NUM_THREADS=%s'
                       % (rows_sample, n, dt, np.__version__, os.environ.get('OPENBLAS_NUM_THREADS', 'unset')))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--n', type=int, default=100000)
    ap.add_argument('--workload', default='box100k')
    ap.add_argument('--cpu-rows', type=int, default=256)
    ap.add_argument('--no-cpu', action='store_true')
    args = ap.parse_args()

    rank = int(os.environ.get('RANK', 0))
    t = synth.workload(args.workload, n=args.n, seed=7)
    n = t.ntraf
    ctx = _lib.Context(int(os.environ.get('LOCAL_RANK', 0)))
    ctx.set_state(t.lat, t.lon, t.trk, t.gs, t.alt, t.vs)

    for _ in range(args.warmup):
        ctx.detect(synth.RPZ, synth.HPZ, synth.TLOOKAHEAD)
    ctx.sync()
    ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        nc, nl = ctx.detect(synth.RPZ, synth.HPZ, synth.TLOOKAHEAD)
        ms.append(ctx.last_timings())
    ctx.sync()
    dt = time.perf_counter() - t0
    pairs = float(n) * n
    value = pairs * args.steps / dt
    pf = np.mean([m['prefilter'] for m in ms]) * 1e-3
    ex = np.mean([m['exact'] for m in ms]) * 1e-3
    ncand = ctx.last_candidates()
    roof = dict(bound='valu', kernel='k_prefilter (fp32 VALU, dominant)',
                achieved=pairs * PF_FLOPS_PER_PAIR / pf / 1e12, peak=FP32_PEAK_TFLOPS,
                unit='TFLOP/s')
    roof['frac'] = roof['achieved'] / roof['peak']
    roof['traffic'] = None
    out = dict(metric='CD pair-evals/s at 100k aircraft', value=value, unit='pair-evals/s',
               n_gpus=args.gpus, steps=args.steps, warmup=args.warmup,
               ms_per_step=dt / args.steps * 1e3, higher_is_better=True, scaling='strong',
               vs_baseline=None, dtype='f64', data='synthetic',
               config=dict(workload='%s N=%d (density-matched box, seed 7)' % (args.workload, n),
                           rpz_m=synth.RPZ, hpz_m=synth.HPZ, tlookahead_s=synth.TLOOKAHEAD,
                           parallelism='dp%d-rows' % args.gpus),
               roofline=roof,
               kernels_ms=dict(order_prep_cull=np.mean([m['prep'] for m in ms]), prefilter=pf * 1e3,
                               exact=ex * 1e3, sort=np.mean([m['sort'] for m in ms])),
               n_conf=nc, n_los=nl, n_candidates=ncand, tile_pairs=ctx.last_tiles(),
               exact_fp64=dict(achieved_tflops=ncand * OPS_PER_PAIR / ex / 1e12 if ex > 0 else None,
                               peak=FP64_PEAK_TFLOPS),
               cd_effective_frac_fp64=value * OPS_PER_PAIR / (FP64_PEAK_TFLOPS * 1e12))
    if rank == 0 and args.gpus == 1 and not args.no_cpu:
        out['cpu_baseline'] = cpu_baseline(t, args.cpu_rows)
        out['speedup_vs_cpu'] = value / out['cpu_baseline']['value']
    if rank == 0:
        print(json.dumps(out))


if __name__ == '__main__':
    main()
