"""Bitwise comparison of two library builds (A/B of a change that must not
move any result): the drop-in detect at box100k (pairs and payload), 40
resident steps at a 20k box with MVP, and a 2048 x 2048 qdrdist matrix.
Each build runs in its own process (BSACCEL_LIB); exit 1 on any difference.
Usage: python tools/ab_bitwise.py bluesky_amd/libA.so bluesky_amd/libB.so"""
import os
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out):
    from bluesky_amd import _lib, geo, resident, statebased, synth
    res = {}
    t = synth.workload('box100k')
    d = statebased.detect_indices(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, with_dcpa=True)
    res.update({'detect_' + k: np.asarray(v) for k, v in d.items()})
    ctx = _lib.Context(0)
    tb = synth.box(20000, 200.0, seed=11)
    sim = resident.ResidentSim(resident.initial_state(tb), resident.params(cd_every=1), ctx=ctx)
    sim.step(40)
    res.update({'sim_' + k: np.asarray(v) for k, v in sim.read().items()})
    ctx.close()
    rng = np.random.default_rng(5)
    la, lo = rng.uniform(-60, 60, 2048), rng.uniform(-180, 180, 2048)
    q, dd = geo.qdrdist_matrix(la, lo, la[::-1].copy(), lo[::-1].copy())
    res['geo_qdr'], res['geo_dist'] = np.asarray(q), np.asarray(dd)
    np.savez(out, **res)


def main():
    if sys.argv[1] == '--run':
        run(sys.argv[2])
        return 0
    tmp = tempfile.mkdtemp()
    files = []
    for k, lib in enumerate(sys.argv[1:3]):
        f = os.path.join(tmp, '%d.npz' % k)
        env = dict(os.environ, BSACCEL_LIB=os.path.abspath(lib), BSACCEL_AB='1')
        subprocess.run([sys.executable, __file__, '--run', f], env=env, check=True, timeout=600)
        files.append(np.load(f))
    a, b = files
    bad = [k for k in a.files if a[k].shape != b[k].shape or a[k].tobytes() != b[k].tobytes()]
    print('arrays compared: %d, differing: %s' % (len(a.files), bad or 'none'))
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main())
