"""One rank's share of a row-sharded CD step on one GPU, repeated (for a
rocprofv3 kernel trace of its launch sequence): bsa_sim_detect_rows of rank
RANK of R on WORKLOAD, REPS times, no stage events.
Usage: python tools/probe_rank.py [WORKLOAD R RANK REPS]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bluesky_amd import _lib, resident, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'global1m'
R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 4
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
t = synth.workload(name)
n = t.ntraf
ctx = _lib.Context(0)
ctx.set_timing_sample(0)
sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx)
rpr = ((n + R - 1) // R + 511) // 512 * 512
rb, re = min(n, rank * rpr), min(n, (rank + 1) * rpr)
for _ in range(3):
    ctx.sim_detect_rows(rb, re)
ctx.sync()
t0 = time.perf_counter()
for _ in range(reps):
    ctx.sim_detect_rows(rb, re)
ctx.sync()
print('%s R=%d rank %d rows %d: %.4f ms per detect (host-synchronised calls)' %
      (name, R, rank, re - rb, (time.perf_counter() - t0) / reps * 1e3))
