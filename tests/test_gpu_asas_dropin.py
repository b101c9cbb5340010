"""GPU: the ASAS.update drop-in (bluesky_amd/asas.py -> bsa_sim_cd) replayed on
the reference's own full-simulator traces (BASELINE.json configs[0] SUPER8 with
MVP, configs[1] 1000.scn with CR OFF, and SUPER8 with stack DEL / CRE between
calls).  A fake ``bs.traf`` / ``bs.traf.asas`` carries each recorded call's
traffic state (what the reference's autopilot / performance model / stack left
before ASAS.update); after ``asas.update(simt)`` every attribute the reference's
ASAS.update sets (asas.py:473-504) must match the recorded one: the pair lists
as callsign tuples (exact, row-major), inconf / tcpamax / qdr / dist / tcpa /
tLOS (1e-9 relative), the resolver's asas.trk / tas / vs / alt / asase / asasn,
resopairs (exact), the four counts (exact) and asas.active (exact wherever the
reference's value does not depend on Python set order)."""
import types

import numpy as np
import pytest

from bluesky_amd import asas as gasas
from oracle import asas as oasas
from tests import util
from tests.test_oracle_trace import traffic_change

pytestmark = pytest.mark.gpu

TRACES = util.golden('trace_*.npz')


def fake_asas(st):
    a = types.SimpleNamespace(swasas=True, tasas=0.0, dtasas=1.0, asaseval=False, noresolst=[], resoofflst=[],
                              swnoreso=False, swresooff=False, priocode=str(st['priocode']), mar=float(st['mar']),
                              R=float(st['rpz']), dh=float(st['hpz']), dtlookahead=float(st['tla']))
    for k in ('Rm', 'dhm', 'vmin', 'vmax', 'vsmin', 'vsmax', 'swresohoriz', 'swresospd', 'swresohdg',
              'swresovert', 'swprio'):
        setattr(a, k, st[k][()])
    a.cd = types.ModuleType('bluesky.traffic.asas.StateBasedCD')
    a.cr = types.ModuleType('bluesky.traffic.asas.' + ('MVP' if str(st['cr']).endswith('MVP') else 'DoNothing'))
    a.resopairs = set()
    a.confpairs_all, a.lospairs_all = [], []
    return a


def load_call(traf, r, ids):
    traf.id = list(ids)
    traf.ntraf = len(ids)
    for k in ('lat', 'lon', 'trk', 'gs', 'alt', 'vs', 'tas', 'gseast', 'gsnorth', 'selalt'):
        setattr(traf, k, np.array(r[k]))
    traf.hdg = np.array(r['trk'])
    traf.ap = types.SimpleNamespace(trk=np.array(r['aptrk']), tas=np.array(r['aptas']), alt=np.array(r['apalt']),
                                    vs=np.array(r['apvs']))


@pytest.mark.parametrize('history', [False, True])
@pytest.mark.parametrize('path', TRACES, ids=[util.case_name(p) for p in TRACES])
def test_asas_update_dropin_matches_reference_trace(ctx, path, history):
    st, calls = util.load_trace(path)
    rpz, tla = float(st['rpz']), float(st['tla'])
    reso = str(st['cr']).endswith('MVP')
    traf = types.SimpleNamespace()
    asas = fake_asas(st)
    dev = gasas.install(asas, traf, ctx=ctx, history=history)
    bk = oasas.Bookkeeping(len(calls[0]['lat']))
    for c, r in enumerate(calls):
        n = len(r['lat'])
        ids = [str(x) for x in r['ids']] if 'ids' in r else ['AC%04d' % k for k in range(n)]
        if c and 'ids' in r:
            deleted, created = traffic_change(calls[c - 1]['ids'], r['ids'])
            if deleted:
                bk.delete(deleted)
            if created:
                bk.create(created)
        load_call(traf, r, ids)
        asas.alt = np.array(r['asas_alt_in'])   # the host's asas.alt before the call (ASAS.create / delete applied)
        asas.update(float(c))
        # the detector's 8-tuple, as callsign tuples
        exp_c = [(ids[i], ids[j]) for i, j in zip(r['ci'].tolist(), r['cj'].tolist())]
        exp_l = [(ids[i], ids[j]) for i, j in zip(r['li'].tolist(), r['lj'].tolist())]
        assert len(asas.confpairs) == len(exp_c) and list(asas.confpairs) == exp_c, c
        assert list(asas.lospairs) == exp_l, c
        assert np.array_equal(asas.inconf, r['inconf'].astype(bool)), c
        for k, sc in (('tcpamax', tla), ('qdr', 360.0), ('dist', rpz), ('tcpa', tla), ('tLOS', tla)):
            ok, msg = util.close(getattr(asas, k), r[k], sc)
            assert ok, 'call %d %s: %s' % (c, k, msg)
        # the resolver's outputs
        if len(exp_c):
            for k, sc in (('trk', 360.0), ('tas', 300.0), ('vs', 20.0), ('alt', 1e4)):
                ok, msg = util.close(getattr(asas, k), r['asas_' + k], sc)
                assert ok, 'call %d asas.%s: %s' % (c, k, msg)
            if reso:
                for k in ('asase', 'asasn'):
                    ok, msg = util.close(getattr(asas, k), r[k], 300.0, rtol=1e-6)
                    assert ok, 'call %d %s: %s' % (c, k, msg)
        # bookkeeping: resopairs, counts, ResumeNav's asas.active
        keep = bk.update(zip(r['ci'], r['cj']), zip(r['li'], r['lj']), r['lat'], r['lon'], r['gseast'],
                         r['gsnorth'], r['trk'], rpz, float(st['Rm']))
        exp_reso = {(ids[i], ids[j]) for i, j in zip(r['reso_i'].tolist(), r['reso_j'].tolist())}
        assert len(asas.resopairs) == len(exp_reso) and set(asas.resopairs) == exp_reso, c
        counts = [len(asas.confpairs_unique), len(asas.lospairs_unique), len(asas.confpairs_all),
                  len(asas.lospairs_all)]
        assert counts == r['counts'].tolist(), c
        assert set(asas.confpairs_unique) == {frozenset(p) for p in exp_c}, c
        amb = np.array(bk.ambiguous(keep), dtype=np.int64)
        una = np.setdiff1d(np.arange(n), amb)
        assert np.array_equal(asas.active[una], r['active'][una]), c
        bk.active[amb] = asas.active[amb]
    if history:
        assert len(asas.confpairs_all) == calls[-1]['counts'][2] and isinstance(asas.confpairs_all, list)
    assert dev.ctx.sim_stats()['cd_calls'] == len(calls)


def test_asas_update_dropin_cadence_reset_and_lists(ctx):
    """The ASAS call cadence (asas.py:474-478: skipped while simt < tasas), an
    ASAS.reset() between calls (a fresh resopairs set re-initialises the device
    bookkeeping), NORESO lists reaching the device MVP, and unsupported CR
    methods failing loudly."""
    st, calls = util.load_trace(util.golden('trace_super8.npz')[0])
    r = calls[3]
    n = len(r['lat'])
    ids = ['AC%04d' % k for k in range(n)]
    traf = types.SimpleNamespace()
    asas = fake_asas(st)
    gasas.install(asas, traf, ctx=ctx)
    load_call(traf, r, ids)
    asas.alt = np.array(r['asas_alt_in'])
    asas.update(0.0)
    first = list(asas.confpairs)
    assert first and asas.tasas == 1.0
    asas.confpairs = None
    asas.update(0.5)                     # before tasas: nothing runs
    assert asas.confpairs is None and asas.tasas == 1.0
    asas.update(1.0)
    assert list(asas.confpairs) == first
    # ASAS.reset(): new containers -> the device bookkeeping starts empty again
    asas.resopairs, asas.confpairs_all, asas.lospairs_all = set(), [], []
    asas.alt = np.array(r['asas_alt_in'])
    asas.update(2.0)
    assert len(asas.confpairs_all) == len({frozenset(p) for p in first})
    # NORESO: nobody avoids AC0000 -> other aircraft's MVP differs from the run without it
    trk0 = asas.trk.copy()
    asas.swnoreso, asas.noresolst = True, ['AC0000']
    asas.alt = np.array(r['asas_alt_in'])
    asas.update(3.0)
    assert not np.array_equal(asas.trk, trk0)
    asas.cr = types.ModuleType('bluesky.traffic.asas.Eby')
    with pytest.raises(NotImplementedError):
        asas.update(4.0)
