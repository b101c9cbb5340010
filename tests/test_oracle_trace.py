"""CPU: the oracle against the reference's own full-simulator traces
(BASELINE.json configs[0] SUPER8 and configs[1] 1000.scn, N = 606).

tests/golden/trace_*.npz were recorded by tools/make_trace.py, which runs the
reference's detached simulator (bluesky.init + Simulation.step) and records
every ASAS.update call (asas.py:473-504): the state the detector read, the
detector outputs, MVP's outputs (MVP.py:14-143), the bookkeeping sets and
ResumeNav's asas.active (asas.py:409-471).  Each call is replayed here through
oracle/statebased.py, oracle/mvp.py and oracle/asas.py: index sets exact,
reals <= 1e-12 relative, counts exact, asas.active exact wherever the
reference's value does not depend on Python set iteration order.
"""
import numpy as np
import pytest

from bluesky_amd import synth
from oracle import asas as oasas
from oracle import mvp as omvp
from oracle import statebased as ocd
from tests import util

TRACES = util.golden('trace_*.npz')


def mvp_params(st):
    return omvp.params_from_settings(float(st['rpz']), float(st['hpz']), float(st['tla']), float(st['mar']),
                                     bool(st['swresohoriz']), bool(st['swresospd']), bool(st['swresohdg']),
                                     bool(st['swresovert']), bool(st['swprio']), str(st['priocode']))


def test_traces_present():
    names = {util.case_name(p) for p in TRACES}
    assert names == {'trace_super8', 'trace_1000scn'}
    st, calls = util.load_trace(util.golden('trace_1000scn.npz')[0])
    assert len(calls[0]['lat']) == 606           # 1000.scn yields 606 aircraft
    st, calls = util.load_trace(util.golden('trace_super8.npz')[0])
    assert len(calls[0]['lat']) == 8 and len(calls[0]['ci']) == 56
    assert len(calls[-1]['reso_i']) == 0 and max(len(c['reso_i']) for c in calls) == 56


@pytest.mark.parametrize('path', TRACES, ids=[util.case_name(p) for p in TRACES])
def test_oracle_matches_reference_trace(path):
    st, calls = util.load_trace(path)
    rpz, hpz, tla = float(st['rpz']), float(st['hpz']), float(st['tla'])
    p = mvp_params(st)
    n = len(calls[0]['lat'])
    bk = oasas.Bookkeeping(n)
    bk.active = calls[0]['active_in'].copy()
    for c, r in enumerate(calls):
        t = synth.Traffic(r['lat'], r['lon'], r['alt'], r['trk'], r['gs'], r['vs'])
        o = ocd.detect_arrays(t, t, rpz, hpz, tla)
        exp = dict(r, tinconf=r['tLOS'])
        util.assert_detect_equal(o, exp, rpz, tla)
        if bool(r['mvp_ran']):
            m = omvp.resolve_arrays(r['ci'], r['cj'], r['qdr'], r['dist'], r['tcpa'], r['tLOS'],
                                    r['gseast'], r['gsnorth'], r['vs'], r['alt'], r['trk'], r['gs'],
                                    r['selalt'], r['apvs'], r['asas_alt_in'].copy(), p)
            for k in ('trk', 'tas', 'vs', 'alt'):
                ok, msg = util.close(m[k], r['asas_' + k], 1.0, rtol=1e-12)
                assert ok, 'call %d asas.%s: %s' % (c, k, msg)
            for k in ('asase', 'asasn'):
                assert np.array_equal(m[k], r[k]), 'call %d %s' % (c, k)
        elif len(r['ci']):   # CR OFF: DoNothing.resolve (DoNothing.py:11-20)
            assert str(st['cr']).endswith('DoNothing')
            for k in ('trk', 'tas', 'vs', 'alt'):
                assert np.array_equal(r['asas_' + k], r['ap' + k]), 'call %d asas.%s' % (c, k)
        keep = bk.update(zip(r['ci'], r['cj']), zip(r['li'], r['lj']), r['lat'], r['lon'], r['gseast'],
                         r['gsnorth'], r['trk'], rpz, float(st['Rm']))
        assert sorted(bk.resopairs) == sorted(zip(r['reso_i'].tolist(), r['reso_j'].tolist())), c
        counts = [len(bk.confpairs_unique), len(bk.lospairs_unique), bk.confpairs_all, bk.lospairs_all]
        assert counts == r['counts'].tolist(), c
        una = np.setdiff1d(np.arange(n), np.array(bk.ambiguous(keep), dtype=np.int64))
        assert np.array_equal(bk.active[una], r['active'][una]), c
        if c + 1 < len(calls):   # nothing outside ASAS.update touches asas.alt / asas.active in these runs
            assert np.array_equal(calls[c + 1]['asas_alt_in'], r['asas_alt'])
            assert np.array_equal(calls[c + 1]['active_in'], r['active'])
