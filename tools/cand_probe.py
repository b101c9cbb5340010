"""Candidates per detect (K1a survivors handed to K1b) against the conflict /
LoS pair counts, for the refine's tightness."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bluesky_amd import _lib, synth  # noqa: E402

ctx = _lib.default_context()
for wl in ('box10k', 'box100k'):
    t = synth.workload(wl)
    ctx.set_state(t.lat, t.lon, t.trk, t.gs, t.alt, t.vs)
    nc, nl = ctx.detect(synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, 0, 0, t.ntraf)
    print(wl, 'conf', nc, 'los', nl, 'candidates', ctx.last_candidates())
