import sys, numpy as np
sys.path.insert(0, '.')
from bluesky_amd import _lib, resident, synth
t = synth.workload(sys.argv[1] if len(sys.argv) > 1 else 'box100k', seed=7)
init = resident.initial_state(t)
for sh, sv in ((800., 60.), (1500., 150.)):
    c = _lib.Context(0)
    c.set_candidate_reuse(True, sh, sv)
    sim = resident.ResidentSim(init, resident.params(), ctx=c)
    hist = []
    for k in range(40):
        sim.step(1)
        hist.append(c.reuse_budget_use())
    print(sh, sv, c.reuse_stats())
    print(' '.join('%.2f/%.2f' % h for h in hist))
    c.close()
