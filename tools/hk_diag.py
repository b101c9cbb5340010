"""Diagnostic: HK (host-known tile-pair list decisions) against the device-
decided run and the full cull, step by step (prints the first difference)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bluesky_amd import _lib, resident, synth  # noqa: E402


def run(ctx, init, p, steps, tile, hk, f=0.75):
    ctx.set_hk(hk, f)
    if tile is None:
        ctx.set_tile_reuse(False)
    else:
        ctx.set_tile_reuse(True, *tile)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    out = []
    for k in range(steps):
        sim.step(1)
        st = sim.stats()
        out.append((sim.read(), ctx.fetch_pairs(st['n_conf'], st['n_los']), ctx.hk_stats(), ctx.tile_reuse_stats()))
    ctx.set_tile_reuse(True)
    ctx.set_hk(True, 0.75)
    return out


def main():
    simdt = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    seq = len(sys.argv) > 2 and sys.argv[2] == 'seq'
    ctx = _lib.Context(0)
    t = synth.box(20000, 300.0, seed=101)
    init = resident.initial_state(t)
    if seq:   # the test file's order: the 0.05 s case first (full cull, then reuse with HK)
        p0 = resident.params(simdt=0.05, cd_every=1, swresohoriz=False)
        run(ctx, init, p0, 24, None, True)
        run(ctx, init, p0, 24, (2016.0, 300.0), True)
    p = resident.params(simdt=simdt, cd_every=1, swresohoriz=False)
    full = run(ctx, init, p, 12, None, True)
    hk = run(ctx, init, p, 12, (2016.0, 300.0), True)
    dev = run(ctx, init, p, 12, (2016.0, 300.0), False)
    for name, r in (('hk', hk), ('device', dev)):
        for k in range(12):
            diff = [f for f in full[k][0] if not np.array_equal(full[k][0][f], r[k][0][f])]
            pd = [f for f in ('ci', 'cj', 'li', 'lj') if not np.array_equal(full[k][1][f], r[k][1][f])]
            print(name, 'step', k, 'n_conf', len(r[k][1]['ci']), 'vs', len(full[k][1]['ci']), 'state diff', diff[:3],
                  'pair diff', pd, r[k][2], r[k][3], flush=True)


if __name__ == '__main__':
    main()
