#!/usr/bin/env python3
"""Capture full-simulator traces from the REFERENCE BlueSky (build container only).

BASELINE.json configs[0] and configs[1] are whole-simulator scenarios, so their
golden vectors come from the reference's own detached simulator
(``bluesky.init('sim-detached')`` + ``bs.sim.step()``), not from calling
``StateBasedCD.detect`` on synthetic inputs.  Every ``ASAS.update`` call that
fires (asas.py:473-504) is wrapped on the instance: the traffic state the
detector reads and the MVP inputs are saved before the call, and the detector
/ resolver outputs, the bookkeeping sets and ``asas.active`` after it.

* ``trace_super8.npz``   -- scenario/ASAS-SUPER8.scn: ``SYN SUPER 8`` restated with
  Python floats (stack/synthetic.py:86-108; the original passes numpy scalars to
  Traffic.create, which crashes in this snapshot), ASAS ON,
  RESO MVP, RMETHH BOTH, RMETHV OFF.  Every ASAS call of the first 360 s
  (approach, resolution, CPA passage and ResumeNav dropping the pairs).
* ``trace_1000scn.npz``  -- scenario/1000.scn (606 aircraft after the duplicate /
  colliding CRE lines), StateBased CD, CR OFF (asas.py:76-77
  defaults).  The first ASAS calls.
* ``trace_super8del.npz`` -- SUPER8 as above with traffic created and deleted
  while the conflicts are being resolved (TrafficArrays create / delete,
  trafficarrays.py:73-118, traffic.py:192-378): ``DEL`` of an aircraft that
  is in other aircraft's resopairs, ``CRE`` of a new one into the conflict,
  then another ``DEL``; every ASAS call of the first 60 s.  Per call the
  callsigns are stored too (``ids``), so a replay can map indices across the
  index shifts of a delete.

Offline shims, all in a scratch run directory outside the repo:
numpy-2 aliases, stub ``zmq`` / ``semver`` modules (bluesky/network/__init__.py
imports them even in detached mode), a ``settings.cfg`` from data/default.cfg
with ``prefer_compiled = False`` and no plugins, navdata symlinks with an empty
``awy.dat`` and an ``apt.zip`` holding an empty ``apt.dat`` (the blobs are not
in the checkout).  The reference is never modified and never leaves this
container; only the arrays are committed (tests/golden/).

Usage:  python tools/make_trace.py   (~1 min)
"""
import os
import shutil
import sys
import tempfile
import types
import zipfile

import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, 'tests', 'golden')


def make_rundir():
    run = tempfile.mkdtemp(prefix='bsref_run_')
    stubs = os.path.join(run, '_stubs')
    for mod in ('zmq', 'semver'):
        os.makedirs(os.path.join(stubs, mod))
        with open(os.path.join(stubs, mod, '__init__.py'), 'w') as f:
            f.write('# offline stub: detached mode never opens a socket\n'
                    'class Context:\n    def __init__(self, *a, **k): pass\n'
                    'def __getattr__(name):\n    return 0\n')
    data = os.path.join(run, 'data')
    os.makedirs(os.path.join(data, 'navdata'))
    for d in ('performance', 'graphics', 'html'):
        os.symlink(os.path.join(REF, 'data', d), os.path.join(data, d))
    shutil.copy(os.path.join(REF, 'data', 'default.cfg'), os.path.join(data, 'default.cfg'))
    nav = os.path.join(REF, 'data', 'navdata')
    for f in os.listdir(nav):
        if f in ('awy.dat', 'apt.zip'):
            continue
        os.symlink(os.path.join(nav, f), os.path.join(data, 'navdata', f))
    open(os.path.join(data, 'navdata', 'awy.dat'), 'w').close()
    with zipfile.ZipFile(os.path.join(data, 'navdata', 'apt.zip'), 'w') as z:
        z.writestr('apt.dat', '')
    os.makedirs(os.path.join(run, 'plugins'))
    shutil.copytree(os.path.join(REF, 'scenario'), os.path.join(run, 'scenario'))
    with open(os.path.join(REF, 'data', 'default.cfg')) as fin, \
            open(os.path.join(run, 'settings.cfg'), 'w') as fout:
        for line in fin:
            if line.startswith('prefer_compiled'):
                line = 'prefer_compiled = False\n'
            elif line.startswith('enabled_plugins'):
                line = 'enabled_plugins = []\n'
            fout.write(line)
    return run, stubs


def init_reference(scnfile=''):
    run, stubs = make_rundir()
    os.chdir(run)
    np.mat = np.asmatrix
    np.int = int
    np.float = float
    np.object = object
    np.str = str
    sys.dont_write_bytecode = True
    sys.path.insert(0, stubs)
    sys.path.insert(0, REF)
    sys.argv = ['BlueSky.py', '--sim', '--detached']
    import bluesky as bs
    bs.init('sim-detached', scnfile=scnfile)
    return bs, run


class Recorder:
    """Wraps bs.traf.asas.update (asas.py:473-504) and records every call that fires."""

    TRAF = ('lat', 'lon', 'trk', 'gs', 'alt', 'vs', 'tas', 'gseast', 'gsnorth', 'selalt')

    def __init__(self, bs):
        self.bs = bs
        self.calls = []
        asas = bs.traf.asas
        self.orig = asas.update
        asas.update = self.update

    def update(self, simt):
        bs = self.bs
        asas, traf = bs.traf.asas, bs.traf
        fires = asas.swasas and simt >= asas.tasas and traf.ntraf > 0
        if not fires:
            return self.orig(simt)
        pre = {k: np.array(getattr(traf, k), dtype=np.float64) for k in self.TRAF}
        for k in ('trk', 'tas', 'alt', 'vs'):
            pre['ap' + k] = np.array(getattr(traf.ap, k), dtype=np.float64)
        pre['asas_alt_in'] = np.array(asas.alt, dtype=np.float64)
        pre['active_in'] = np.array(asas.active, dtype=bool)
        ids = list(traf.id)
        reso_in = sorted(asas.resopairs)
        self.orig(simt)
        idx = {k: i for i, k in enumerate(ids)}

        def pairs(lst):  # ids of deleted aircraft (still in resopairs until ResumeNav) -> -1
            a = np.array([(idx.get(p, -1), idx.get(q, -1)) for p, q in lst], dtype=np.int64).reshape(-1, 2)
            return a[:, 0], a[:, 1]

        rec = dict(simt=simt, ids=np.array(ids, dtype='U16'), **pre)
        rec['ci'], rec['cj'] = pairs(asas.confpairs)
        rec['li'], rec['lj'] = pairs(asas.lospairs)
        rec['inconf'] = np.array(asas.inconf, dtype=bool)
        rec['tcpamax'] = np.array(asas.tcpamax, dtype=np.float64)
        for k in ('qdr', 'dist', 'tcpa', 'tLOS'):
            rec[k] = np.array(getattr(asas, k), dtype=np.float64)
        for k in ('trk', 'tas', 'vs', 'alt'):
            rec['asas_' + k] = np.array(getattr(asas, k), dtype=np.float64)
        for k in ('asase', 'asasn'):
            rec[k] = np.array(getattr(asas, k))
        rec['mvp_ran'] = bool(asas.confpairs) and asas.cr.__name__.endswith('MVP')
        rec['active'] = np.array(asas.active, dtype=bool)
        rec['reso_in_i'], rec['reso_in_j'] = pairs(reso_in)
        rec['reso_i'], rec['reso_j'] = pairs(sorted(asas.resopairs))
        rec['counts'] = np.array([len(asas.confpairs_unique), len(asas.lospairs_unique),
                                  len(asas.confpairs_all), len(asas.lospairs_all)], dtype=np.int64)
        self.calls.append(rec)


def asas_settings(asas):
    return dict(rpz=asas.R, hpz=asas.dh, tla=asas.dtlookahead, mar=asas.mar, Rm=asas.Rm, dhm=asas.dhm,
                vmin=asas.vmin, vmax=asas.vmax, vsmin=asas.vsmin, vsmax=asas.vsmax,
                swresohoriz=asas.swresohoriz, swresospd=asas.swresospd, swresohdg=asas.swresohdg,
                swresovert=asas.swresovert, swprio=asas.swprio, priocode=str(asas.priocode),
                dtasas=asas.dtasas)


PAIR_KEYS = ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tLOS', 'li', 'lj', 'reso_in_i', 'reso_in_j',
             'reso_i', 'reso_j')
SCALAR_KEYS = ('simt', 'mvp_ran')


def save(name, calls, settings):
    """Per-aircraft arrays stacked as [call, aircraft] when every call has the
    same traffic, else (create / delete) concatenated like the pair arrays;
    pair arrays of all calls concatenated, with ``<key>_off`` offsets
    [ncalls + 1] (conflict-pair keys share ``ci_off``, LoS keys ``li_off``,
    resopairs ``reso_i_off`` / ``reso_in_i_off``)."""
    d = {'ncalls': np.array(len(calls))}
    for k, v in settings.items():
        d['set_' + k] = np.array(v)
    same_n = len({len(rec['lat']) for rec in calls}) == 1
    for k in calls[0]:
        if k == 'ids' and same_n:
            continue
        vals = [np.asarray(rec[k]) for rec in calls]
        if k in PAIR_KEYS or (not same_n and k not in SCALAR_KEYS):
            d[k] = np.concatenate(vals)
            d[k + '_off'] = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.int64)
        else:
            d[k] = np.stack(vals)
    np.savez_compressed(os.path.join(OUT, name), **d)


def run_super8(bs, seconds=360.0):
    """ASAS-SUPER8.scn with SYN SUPER 8 restated in Python floats."""
    from bluesky import stack
    from bluesky.tools.aero import ft
    traf = bs.traf
    numac, distance, alt, spd = 8, 0.50, 20000 * ft, 200
    for i in range(numac):
        angle = 2 * np.pi / numac * i
        traf.create(acid='SUP' + str(i), actype='SUPER', aclat=float(distance * -np.cos(angle)),
                    aclon=float(distance * np.sin(angle)), achdg=float(360.0 - 360.0 / numac * i),
                    acalt=float(alt), acspd=float(spd))
    for cmd in ('ASAS ON', 'RESO MVP', 'RMETHH BOTH', 'RMETHV OFF'):
        stack.stack(cmd)
    rec = Recorder(bs)
    nsteps = int(round(seconds / bs.sim.simdt))
    bs.sim.step()
    bs.sim.fastforward()
    for _ in range(nsteps):
        bs.sim.step()
    settings = asas_settings(traf.asas)
    settings['cd'] = traf.asas.cd.__name__
    settings['cr'] = traf.asas.cr.__name__
    return rec.calls, settings


def run_super8del(bs, seconds=60.0):
    """SUPER8 with a delete, a create into the conflict and another delete."""
    from bluesky import stack
    from bluesky.tools.aero import ft
    traf = bs.traf
    numac, distance, alt, spd = 8, 0.50, 20000 * ft, 200
    for i in range(numac):
        angle = 2 * np.pi / numac * i
        traf.create(acid='SUP' + str(i), actype='SUPER', aclat=float(distance * -np.cos(angle)),
                    aclon=float(distance * np.sin(angle)), achdg=float(360.0 - 360.0 / numac * i),
                    acalt=float(alt), acspd=float(spd))
    for cmd in ('ASAS ON', 'RESO MVP', 'RMETHH BOTH', 'RMETHV OFF'):
        stack.stack(cmd)
    rec = Recorder(bs)
    events = {int(round(6.5 / bs.sim.simdt)): lambda: traf.delete(traf.id.index('SUP2')),
              int(round(9.5 / bs.sim.simdt)): lambda: traf.create(acid='NEW1', actype='SUPER', aclat=0.05,
                                                                     aclon=-0.3, achdg=80.0,
                                                                     acalt=float(alt), acspd=float(spd)),
              int(round(14.5 / bs.sim.simdt)): lambda: traf.delete(traf.id.index('SUP5')),
              int(round(20.5 / bs.sim.simdt)): lambda: traf.delete(np.array([traf.id.index('SUP0'),
                                                                             traf.id.index('NEW1')]))}
    nsteps = int(round(seconds / bs.sim.simdt))
    bs.sim.step()
    bs.sim.fastforward()
    for k in range(nsteps):
        if k in events:
            events[k]()
        bs.sim.step()
    settings = asas_settings(traf.asas)
    settings['cd'] = traf.asas.cd.__name__
    settings['cr'] = traf.asas.cr.__name__
    return rec.calls, settings


def run_1000(bs, ncalls=8):
    rec = Recorder(bs)
    bs.sim.step()
    bs.sim.fastforward()
    while len(rec.calls) < ncalls:
        bs.sim.step()
    settings = asas_settings(bs.traf.asas)
    settings['cd'] = bs.traf.asas.cd.__name__
    settings['cr'] = bs.traf.asas.cr.__name__
    return rec.calls, settings


def main():
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1] if len(sys.argv) > 1 else 'all'
    if which in ('all', 'super8'):
        if which == 'all':   # one reference process per scenario (bluesky is a singleton)
            import subprocess
            for w in ('super8', '1000', 'super8del'):
                subprocess.run([sys.executable, os.path.abspath(__file__), w], check=True)
            return
        bs, run = init_reference()
        calls, st = run_super8(bs)
        save('trace_super8.npz', calls, st)
        print('trace_super8: %d ASAS calls, conf per call %s, mvp %s' % (
            len(calls), [len(c['ci']) for c in calls], [int(c['mvp_ran']) for c in calls]))
        shutil.rmtree(run, ignore_errors=True)
    elif which == 'super8del':
        bs, run = init_reference()
        calls, st = run_super8del(bs)
        save('trace_super8del.npz', calls, st)
        print('trace_super8del: %d ASAS calls, N %s, conf %s' % (
            len(calls), [len(c['lat']) for c in calls], [len(c['ci']) for c in calls]))
        shutil.rmtree(run, ignore_errors=True)
    elif which == '1000':
        bs, run = init_reference(scnfile=os.path.join('scenario', '1000.scn'))
        calls, st = run_1000(bs)
        save('trace_1000scn.npz', calls, st)
        print('trace_1000scn: %d ASAS calls, N %s, conf %s, los %s' % (
            len(calls), [len(c['lat']) for c in calls], [len(c['ci']) for c in calls],
            [len(c['li']) for c in calls]))
        shutil.rmtree(run, ignore_errors=True)


if __name__ == '__main__':
    main()
