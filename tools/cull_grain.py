"""Host estimate of the prefilter's stage-1 tests against the row granularity
of its box cull: rows in slices of GR, columns in sub-groups of GC, every
(slice, sub-group) pair whose boxes may interact counted as GR x GC tests
(midpoint stage 1, Hilbert order of tools/cull_sim2.py).  The device sweeps
64-row slices x 8-column sub-groups.
Usage: PYTHONPATH=. python tools/cull_grain.py [WORKLOAD]"""
import sys
import types

import numpy as np

from bluesky_amd import synth

src = open('tools/cull_sim2.py').read().replace("main(sys.argv[1] if len(sys.argv) > 1 else 'box100k')", "")
cs = types.ModuleType('cull_sim2')
exec(src, cs.__dict__)

wl = sys.argv[1] if len(sys.argv) > 1 else 'box100k'
t = synth.workload(wl, seed=7)
R, H, T = 9260., 304.8, 300.
lat, lon = np.radians(t.lat), np.radians(t.lon)
sl, cl, so, co = np.sin(lat), np.cos(lat), np.sin(lon), np.cos(lon)
u, v = t.gs * np.sin(np.radians(t.trk)), t.gs * np.cos(np.radians(t.trk))
ht = 0.5 * T
f = ht / 6371000.0
P = np.stack([cl * co + f * (-u * so - v * sl * co), cl * so + f * (u * co - v * sl * so), sl + f * (v * cl)], 1)
ag = np.abs(t.gs) + 0.5e-3
cmax = (R + (ag + 400.5e-3 + 400) * T) * (1 + 1e-5) / 6.35e6
kb = np.pi / 2 + (1 + np.pi / 2) / (cl - cmax)
s = ((0.5 * R + ag * ht) * (1 + 1e-5) + 0.012 * (0.5 * R + ag * T) + ag * ht * kb * cmax) / 6.3e6 \
    + 0.25 * cmax ** 2 + 1e-6
am = t.alt + t.vs * ht
h = (0.5 * H + (np.abs(t.vs) + 1.5e-6) * ht) * (1 + 1e-5) + 0.5 + 1e-6 * np.abs(am)
lo, hi = am - h, am + h
mn, mx = P.min(0), P.max(0)
span = (mx - mn).max()
q = np.stack([cs.quant(P[:, k], mn[k], mn[k] + span, 16) for k in range(3)] +
             [cs.quant(am, am.min(), am.min() + span * 6371000.0 / 500., 16)], 1)
o = np.argsort(cs.hilbert(q, 16), kind='stable')
P, s, lo, hi = P[o], s[o], lo[o], hi[o]
for gr, gc in ((64, 8), (32, 8), (16, 8), (8, 8)):
    print('%s rows x %d, columns x %d: %.3e stage-1 tests' % (wl, gr, gc, cs.count(P, s, lo, hi, gr, gc)), flush=True)
