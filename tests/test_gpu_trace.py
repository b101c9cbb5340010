"""GPU parity on the reference's own full-simulator traces: BASELINE.json
configs[0] (scenario/ASAS-SUPER8.scn, StateBased CD + MVP, RMETHH BOTH) and
configs[1] (scenario/1000.scn, N = 606, StateBased CD, CR OFF), and SUPER8
with stack DEL / CRE commands mid-run (trace_super8del: Traffic.delete /
create between calls, replayed with bsa_sim_delete / bsa_sim_create).

tests/golden/trace_*.npz hold, per ASAS.update call of the reference's
detached simulator (tools/make_trace.py), the state the detector read and the
reference's outputs.  Three paths are replayed through libbsaccel:

* the drop-in modules a BlueSky user registers -- ``statebased.detect``
  (StateBasedCD.py:7-103, id tuples) and ``mvp.resolve(asas, traf)``
  (MVP.py:14-143) on SimpleNamespace stand-ins for ``bs.traf`` / ``bs.traf.asas``;
* the GPU-resident step with ``resume_nav`` (asas.py:409-504): the state of each
  call is written with ``bsa_sim_update`` (the host simulator's autopilot /
  performance model ran in between), one step runs detect -> resolver (MVP for
  SUPER8, the default CR OFF = DoNothing.resolve for 1000.scn) -> bookkeeping
  -> ResumeNav on the device, and resopairs, the four pair counts,
  asas.trk/tas/vs/alt and asas.active are compared with the reference's.

Pair lists exact, reals <= 1e-9 relative, counts exact, asas.active exact where
the reference's value does not depend on Python set order (oracle/asas.py).
"""
import types

import numpy as np
import pytest

from bluesky_amd import mvp, resident, statebased
from oracle import asas as oasas
from tests import util
from tests.test_oracle_trace import traffic_change

pytestmark = pytest.mark.gpu

TRACES = util.golden('trace_*.npz')


def traf_ns(r):
    n = len(r['lat'])
    t = types.SimpleNamespace(ntraf=n, id=['AC%04d' % k for k in range(n)])
    for k in ('lat', 'lon', 'trk', 'gs', 'alt', 'vs', 'tas', 'gseast', 'gsnorth', 'selalt'):
        setattr(t, k, np.array(r[k]))
    t.ap = types.SimpleNamespace(vs=np.array(r['apvs']))
    return t


def asas_ns(st, r, res):
    a = types.SimpleNamespace(swasas=True, asaseval=False, noresolst=[], resoofflst=[], swnoreso=False,
                              swresooff=False, mar=float(st['mar']), priocode=str(st['priocode']))
    for k in ('Rm', 'dhm', 'vmin', 'vmax', 'vsmin', 'vsmax', 'swresohoriz', 'swresospd', 'swresohdg',
              'swresovert', 'swprio'):
        setattr(a, k, st[k][()])
    a.dtlookahead = float(st['tla'])
    a.confpairs, a.lospairs, a.inconf, a.tcpamax, a.qdr, a.dist, a.tcpa, a.tLOS = res
    a.alt = np.array(r['asas_alt_in'])
    return a


@pytest.mark.parametrize('path', TRACES, ids=[util.case_name(p) for p in TRACES])
def test_dropin_detect_and_mvp_match_reference_trace(ctx, path):
    st, calls = util.load_trace(path)
    rpz, hpz, tla = float(st['rpz']), float(st['hpz']), float(st['tla'])
    for c, r in enumerate(calls):
        if c > 40 and not len(r['ci']) and c % 10:   # the quiet tail of SUPER8: every 10th call
            continue
        traf = traf_ns(r)
        res = statebased.detect(traf, traf, rpz, hpz, tla)
        assert len(res) == 8
        idx = {k: i for i, k in enumerate(traf.id)}
        got = dict(ci=[idx[a] for a, _ in res[0]], cj=[idx[b] for _, b in res[0]],
                   li=[idx[a] for a, _ in res[1]], lj=[idx[b] for _, b in res[1]], inconf=res[2],
                   tcpamax=res[3], qdr=res[4], dist=res[5], tcpa=res[6], tinconf=res[7])
        util.assert_detect_equal(got, dict(r, tinconf=r['tLOS']), rpz, tla)
        if bool(r['mvp_ran']):
            asas = asas_ns(st, r, res)
            mvp.resolve(asas, traf, ctx=ctx)            # device-resident pairs of the detect above
            for k, s in (('trk', 360.0), ('tas', 300.0), ('vs', 20.0), ('alt', 1e4)):
                ok, msg = util.close(asas.__dict__[k], r['asas_' + k], s)
                assert ok, 'call %d asas.%s: %s' % (c, k, msg)
            for k in ('asase', 'asasn'):
                ok, msg = util.close(asas.__dict__[k], r[k], 300.0, rtol=1e-6)  # float32 (MVP.py:117-118)
                assert ok, 'call %d %s: %s' % (c, k, msg)
            # the same resolve on host pairs (another CD produced them): bsa_set_pairs path
            asas2 = asas_ns(st, r, (list(res[0]),) + tuple(res[1:]))
            mvp.resolve(asas2, traf, ctx=ctx)
            for k in ('trk', 'tas', 'vs', 'alt'):
                assert np.array_equal(asas2.__dict__[k], asas.__dict__[k]), k


def sim_state(r, sel):
    """bsa_sim_state of aircraft ``sel`` of trace call ``r``."""
    g = lambda k: np.array(r[k])[sel]
    m = len(g('lat'))
    return dict(lat=g('lat'), lon=g('lon'), alt=g('alt'), tas=g('tas'), hdg=g('trk'), vs=g('vs'), gs=g('gs'),
                trk=g('trk'), gseast=g('gseast'), gsnorth=g('gsnorth'), ap_trk=g('aptrk'), ap_tas=g('aptas'),
                ap_alt=g('apalt'), ap_vs=g('apvs'), selalt=g('selalt'), bank=np.full(m, np.radians(25.)),
                eps=np.full(m, 0.01), accel=np.full(m, 0.5), asas_alt=g('asas_alt_in'))


@pytest.mark.parametrize('path', TRACES, ids=[util.case_name(p) for p in TRACES])
def test_resident_resume_nav_matches_reference_trace(ctx, path):
    st, calls = util.load_trace(path)
    reso = str(st['cr']).endswith('MVP')
    r0 = calls[0]
    n = len(r0['lat'])
    init = sim_state(r0, slice(None))
    p = resident.params(rpz=float(st['rpz']), hpz=float(st['hpz']), tla=float(st['tla']), mar=float(st['mar']),
                        reso=reso, swresohoriz=bool(st['swresohoriz']), swresospd=bool(st['swresospd']),
                        swresohdg=bool(st['swresohdg']), swresovert=bool(st['swresovert']),
                        resume_nav=True, simdt=0.05)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    bk = oasas.Bookkeeping(n)
    assert not r0['active_in'].any()
    for c, r in enumerate(calls):
        n = len(r['lat'])
        if c and 'ids' in r:   # stack DEL / CRE between the calls
            deleted, created = traffic_change(calls[c - 1]['ids'], r['ids'])
            if deleted:
                sim.delete(deleted)
                bk.delete(deleted)
            if created:
                sim.create(sim_state(r, slice(n - created, n)))
                bk.create(created)
            i, j = sim.resopairs()
            live = sorted(set((a, b) for a, b in zip(r['reso_in_i'].tolist(), r['reso_in_j'].tolist()) if a >= 0))
            assert sorted(set(zip(i.tolist(), j.tolist()))) == live, c
        sim.update(lat=r['lat'], lon=r['lon'], trk=r['trk'], gs=r['gs'], alt=r['alt'], vs=r['vs'], tas=r['tas'],
                   gseast=r['gseast'], gsnorth=r['gsnorth'], selalt=r['selalt'], ap_vs=r['apvs'],
                   ap_trk=r['aptrk'], ap_tas=r['aptas'], ap_alt=r['apalt'])
        sim.step(1)
        assert sim.stats()['n_conf'] == len(r['ci']) and sim.stats()['n_los'] == len(r['li']), c
        keep = bk.update(zip(r['ci'], r['cj']), zip(r['li'], r['lj']), r['lat'], r['lon'], r['gseast'],
                         r['gsnorth'], r['trk'], float(st['rpz']), float(st['Rm']))
        i, j = sim.resopairs()
        assert sorted(zip(i.tolist(), j.tolist())) == sorted(zip(r['reso_i'].tolist(), r['reso_j'].tolist())), c
        s = sim.asas_stats()
        assert [s['confpairs_unique'], s['lospairs_unique'], s['confpairs_all'], s['lospairs_all']] == \
            r['counts'].tolist(), c
        got = sim.read()
        amb = np.array(bk.ambiguous(keep), dtype=np.int64)
        una = np.setdiff1d(np.arange(n), amb)
        assert np.array_equal(got['active'][una], r['active'][una]), c
        bk.active[amb] = got['active'][amb]   # the device's order-free outcome
        for k, sc in (('trk', 360.0), ('tas', 300.0), ('vs', 20.0), ('alt', 1e4)):
            ok, msg = util.close(got['asas_' + k], r['asas_' + k], sc)
            assert ok, 'call %d asas.%s: %s' % (c, k, msg)
    assert sim.stats()['cd_calls'] == len(calls)
