"""Per-rank share of the WHOLE sharded step on one GPU:
the resident step of one rank of R -- its detect (own tiles, halo plan, halo
tiles: bsa_sim_detect_rows' one-GPU halo mode), K2, K3 and K4' on its home
rows -- with no collective (bsa_sim_probe_rank), timed as one batch of STEPS
steps (one host synchronisation at its end, no stage events) after SETTLE
untimed ones (the device at steady clocks, as bench.py's --settle).  Collectives
(box all-gather, halo send / recv, gate all-reduce) are excluded: they need
the 8-GPU node.  Prints every rank's ms per step and the slowest.
Usage: python tools/probe_step.py [WORKLOAD [R [STEPS [RANK [SETTLE]]]]]  (RANK: that rank of R
only, -1 all; SETTLE default 200)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bluesky_amd import _lib, resident, synth  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else 'global1m'
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    only = int(sys.argv[4]) if len(sys.argv) > 4 and int(sys.argv[4]) >= 0 else None
    settle = int(sys.argv[5]) if len(sys.argv) > 5 else 200
    t = synth.workload(name)
    ctx = _lib.Context(0)
    ctx.set_timing_sample(0)
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx)
    out = {}
    for ranks in sorted({1, R}) if only is None else [R]:
        per = []
        for r in range(ranks) if only is None else [only]:
            ctx.sim_probe_rank(r, ranks)
            sim.step(5)                      # warm-up: this rank's plan / lists / buffers
            ctx.sync()
            if settle > 0:
                sim.step(settle)
                ctx.sync()
            t0 = time.perf_counter()
            sim.step(steps)
            ctx.sync()
            per.append((time.perf_counter() - t0) / steps * 1e3)
            st = sim.stats()
            print('%s R=%d rank %d rows [%d, %d): %.4f ms per step' % (name, ranks, r, st['row_begin'],
                                                                      st['row_end'], per[-1]), flush=True)
        out['R=%d' % ranks] = dict(slowest_ms=max(per), per_rank_ms=[round(x, 4) for x in per])
    ctx.sim_probe_rank(0, 1)
    print(json.dumps(dict(workload=name, steps=steps, settle=settle, **out)), flush=True)


if __name__ == '__main__':
    main()
