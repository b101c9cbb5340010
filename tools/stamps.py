"""Prefilter phase stamps (diagnostic build): host-path detects on box100k."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bluesky_amd import _lib, synth  # noqa: E402

t = synth.workload('box100k', seed=7)
ctx = _lib.Context(0)
ctx.set_state(t.lat, t.lon, t.trk, t.gs, t.alt, t.vs)
for _ in range(3):
    ctx.detect(synth.RPZ, synth.HPZ, synth.TLOOKAHEAD)
print('timings', ctx.last_timings(), 'tiles', ctx.last_tiles(), 'cand', ctx.last_candidates())
