"""Work of the row-sharded resident step on ONE GPU: `world` ranks of the
in-process group transport (one thread + context each) step the same sim.
Run under `rocprofv3 --kernel-trace --stats`, the per-kernel totals are the
summed work of all ranks, to compare with world 1 (how much of the detect is
replicated or inflated by the sharding).  Ranks share the GPU, so the wall time
printed here is NOT the multi-GPU step time.
Usage: python tools/group_probe.py WORKLOAD WORLD [STEPS]"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bluesky_amd import _lib, resident, synth  # noqa: E402


def main():
    name, world = sys.argv[1], int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    t = synth.workload(name)
    init = resident.initial_state(t)
    p = resident.params(cd_every=1)
    group = _lib.Group(world)
    ctxs = [_lib.Context(0) for _ in range(world)]
    out = [None] * world

    def body(r):
        sim = resident.ResidentSim(init, p, ctx=ctxs[r], rank=r, world=world, group=group)
        sim.step(2)
        ctxs[r].sync()
        t0 = time.perf_counter()
        sim.step(steps)
        ctxs[r].sync()
        st = sim.stats()
        out[r] = (time.perf_counter() - t0, st['row_end'] - st['row_begin'], st['n_conf'])

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(600)
    for r, o in enumerate(out):
        print('%s world %d rank %d: %s' % (name, world, r, o), flush=True)
    for c in ctxs:
        c.close()
    group.close()


if __name__ == '__main__':
    main()
