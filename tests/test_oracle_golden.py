"""CPU: the oracle restatement against the reference's golden vectors.

The vectors were captured by running the reference itself (tools/make_golden.py,
which also asserted bitwise equality at capture time).  Here the check is
exact for index sets and <= 1e-12 relative for reals, so it also holds on a
host whose numpy/libm dispatch differs by an ULP from the capture host.
"""
import numpy as np
import pytest

from oracle import kinematics as okin
from oracle import mvp as omvp
from oracle import statebased as ocd
from tests import util

CD = util.golden('cd_*.npz')
MVP = util.golden('mvp_*.npz')
KIN = util.golden('kin_*.npz')
KWIK = util.golden('cdkwik_*.npz')
ASAS = util.golden('asas_*.npz')


def test_fixtures_present():
    assert len(CD) >= 9 and len(MVP) >= 5 and len(KIN) >= 3 and len(KWIK) >= 6 and len(ASAS) >= 3


@pytest.mark.parametrize('path', ASAS, ids=[util.case_name(p) for p in ASAS])
def test_oracle_asas_bookkeeping_matches_reference(path):
    """ASAS.update's resopairs / unique / cumulative bookkeeping and ResumeNav's
    asas.active (asas.py:409-504), replayed over the reference's recorded calls.
    active is compared where the reference's result does not depend on set
    iteration order (aircraft whose resopairs agree, oracle/asas.py)."""
    from oracle import asas as oasas
    z = np.load(path)
    n = int(z['n'])
    bk = oasas.Bookkeeping(n)
    for k in range(int(z['ncalls'])):
        keep = bk.update(zip(z['ci%d' % k], z['cj%d' % k]), zip(z['li%d' % k], z['lj%d' % k]),
                         z['lat%d' % k], z['lon%d' % k], z['gseast'], z['gsnorth'], z['trk'],
                         float(z['rpz']), float(z['rm']))
        assert sorted(bk.resopairs) == list(zip(z['reso_i%d' % k].tolist(), z['reso_j%d' % k].tolist())), k
        counts = [len(bk.confpairs_unique), len(bk.lospairs_unique), bk.confpairs_all, bk.lospairs_all]
        assert counts == z['counts%d' % k].tolist(), k
        amb = np.array(bk.ambiguous(keep), dtype=np.int64)
        assert np.array_equal(amb, z['ambiguous%d' % k]), k
        una = np.setdiff1d(np.arange(n), amb)
        assert np.array_equal(bk.active[una], z['active%d' % k][una]), k


@pytest.mark.parametrize('path', KWIK, ids=[util.case_name(p) for p in KWIK])
def test_oracle_kwik_matches_reference(path):
    """Opt-in KWIK variant: kwikqdrdist_matrix swapped into the reference's detect."""
    own, intr, z = util.load_cd(path)
    o = ocd.detect_arrays(own, intr, float(z['rpz']), float(z['hpz']), float(z['tla']),
                          budget_bytes=256 << 20, kwik=True)
    for k in ('ci', 'cj', 'li', 'lj'):
        assert np.array_equal(o[k], z[k]), k
    assert np.array_equal(o['inconf'], z['inconf'])
    for k, s in (('qdr', 360.0), ('dist', 1e4), ('tcpa', 300.0), ('tinconf', 300.0),
                 ('tcpamax', 300.0)):
        ok, msg = util.close(o[k], z[k], s, rtol=1e-12)
        assert ok, '%s: %s' % (k, msg)


@pytest.mark.parametrize('path', CD, ids=[util.case_name(p) for p in CD])
def test_oracle_detect_matches_reference(path):
    own, intr, z = util.load_cd(path)
    o = ocd.detect_arrays(own, intr, float(z['rpz']), float(z['hpz']), float(z['tla']),
                          budget_bytes=256 << 20)
    for k in ('ci', 'cj', 'li', 'lj'):
        assert np.array_equal(o[k], z[k]), k
    assert np.array_equal(o['inconf'], z['inconf'])
    for k, s in (('qdr', 360.0), ('dist', 1e4), ('tcpa', 300.0), ('tinconf', 300.0),
                 ('tcpamax', 300.0)):
        ok, msg = util.close(o[k], z[k], s, rtol=1e-12)
        assert ok, '%s: %s' % (k, msg)


def test_oracle_tuple_contract():
    own, intr, z = util.load_cd(util.golden('cd_box64.npz')[0])
    res = ocd.detect(own.as_dict(), own.as_dict(), float(z['rpz']), float(z['hpz']), float(z['tla']))
    assert len(res) == 8
    confpairs, lospairs = res[0], res[1]
    assert confpairs and isinstance(confpairs[0], tuple) and isinstance(confpairs[0][0], str)
    assert [(own.id.index(a), own.id.index(b)) for a, b in confpairs] == list(zip(z['ci'], z['cj']))


MODES = ['default', 'spd', 'hdg', 'vert', 'hv', 'ff1', 'ff2', 'ff3', 'lay1', 'lay2', 'noreso', 'resooff']
MODE_SW = {
    'default': (True, False, False, False, False, 'FF1'), 'spd': (True, True, False, False, False, 'FF1'),
    'hdg': (True, False, True, False, False, 'FF1'), 'vert': (False, False, False, True, False, 'FF1'),
    'hv': (False, False, False, False, False, 'FF1'), 'ff1': (False, False, False, False, True, 'FF1'),
    'ff2': (False, False, False, False, True, 'FF2'), 'ff3': (False, False, False, False, True, 'FF3'),
    'lay1': (False, False, False, False, True, 'LAY1'), 'lay2': (False, False, False, False, True, 'LAY2'),
    'noreso': (False, False, False, False, False, 'FF1'), 'resooff': (False, False, False, False, False, 'FF1'),
}


def mvp_args(z, mode):
    n = len(z['alt'])
    p = omvp.params_from_settings(float(z['rpz']), float(z['hpz']), float(z['tla']), float(z['mar']),
                                  *MODE_SW[mode])
    noreso = np.isin(np.arange(n), z['noreso_idx']) if mode == 'noreso' else None
    resooff = np.isin(np.arange(n), z['resooff_idx']) if mode == 'resooff' else None
    return p, noreso, resooff


@pytest.mark.parametrize('path', MVP, ids=[util.case_name(p) for p in MVP])
def test_oracle_mvp_matches_reference(path):
    z = dict(np.load(path, allow_pickle=False))
    for mode in MODES:
        p, noreso, resooff = mvp_args(z, mode)
        o = omvp.resolve_arrays(z['ci'], z['cj'], z['qdr'], z['dist'], z['tcpa'], z['tLOS'],
                                z['gseast'], z['gsnorth'], z['vs'], z['alt'], z['trk'], z['gs'],
                                z['selalt'], z['apvs'], z['asasalt'].copy(), p, noreso, resooff)
        for k in ('trk', 'tas', 'vs', 'alt', 'asase', 'asasn'):
            ok, msg = util.close(o[k], z['%s__%s' % (mode, k)], 1.0, rtol=1e-12)
            assert ok, '%s/%s: %s' % (mode, k, msg)


@pytest.mark.parametrize('path', KIN, ids=[util.case_name(p) for p in KIN])
def test_oracle_kinematics_matches_reference(path):
    z = dict(np.load(path, allow_pickle=False))
    s = {k: z[k] for k in ('lat', 'lon', 'alt', 'tas', 'hdg', 'vs', 'ptas', 'phdg', 'palt', 'pvs',
                           'bank', 'eps', 'accel')}
    if int(z['winddim']) == 2:   # 2-D field (windfield.py:158-179) at the pre-step positions
        vn, ve = okin.windfield_2d(z['lat'], z['lon'], z['wlat'], z['wlon'], z['wvnorth'], z['wveast'])
        assert util.close(vn, z['windnorth'], 1.0, rtol=1e-12)[0] and util.close(ve, z['windeast'], 1.0, rtol=1e-12)[0]
        o = okin.step(s, float(z['dt']), 1, vn, ve)
    else:
        o = okin.step(s, float(z['dt']), int(z['winddim']), float(z['windnorth']), float(z['windeast']))
    for k in ('ax', 'delspd', 'tas', 'cas', 'M', 'hdg', 'swhdgsel', 'swaltsel', 'az', 'vs',
              'gsnorth', 'gseast', 'gs', 'trk', 'alt', 'lat', 'lon', 'coslat'):
        ok, msg = util.close(np.asarray(o[k], dtype=np.float64),
                             np.asarray(z['out_' + k], dtype=np.float64), 1.0, rtol=1e-12)
        assert ok, '%s: %s' % (k, msg)


GEO = util.golden('geo_*.npz')


@pytest.mark.parametrize('path', GEO, ids=[util.case_name(p) for p in GEO])
def test_oracle_geo_matches_reference(path):
    """Standalone geo.qdrdist_matrix / kwikqdrdist_matrix (geo.py:110-162,
    347-363), outer (row vectors) and pairwise (1-D) operands."""
    from oracle import geo as ogeo
    z = np.load(path)
    fn, mode = str(z['fn']), str(z['mode'])
    f = {('qdrdist', 'outer'): ogeo.qdrdist_outer, ('qdrdist', 'pairwise'): ogeo.qdrdist_pairwise,
         ('kwik', 'outer'): ogeo.kwik_outer, ('kwik', 'pairwise'): ogeo.kwik_pairwise}[fn, mode]
    qdr, dist = f(z['lat1'], z['lon1'], z['lat2'], z['lon2'])
    for k, got in (('qdr', qdr), ('dist', dist)):
        exp = z[k].ravel()
        ok, msg = util.close(np.asarray(got).ravel(), exp, 0.0, rtol=1e-12)
        assert ok, '%s: %s' % (k, msg)


def test_geo_fixtures_present():
    kinds = {(str(np.load(p)['fn']), str(np.load(p)['mode'])) for p in GEO}
    assert kinds == {('qdrdist', 'outer'), ('qdrdist', 'pairwise'), ('kwik', 'outer'), ('kwik', 'pairwise')}


LIMITS = util.golden('limits_*.npz')


@pytest.mark.parametrize('path', LIMITS, ids=[util.case_name(p) for p in LIMITS])
def test_oracle_openap_limits_matches_reference(path):
    """OpenAP.limits (perfoap.py:185-209) as Pilot.applylimits applies it."""
    z = np.load(path)
    env = {k: z[k] for k in ('hmax', 'vmin', 'vmax', 'vsmin', 'vsmax', 'axmax')}
    t, v, h = okin.openap_limits(z['tas'], z['vs'], z['h'], z['ax'], env)
    for k, got in (('tas', t), ('vs', v), ('alt', h)):
        ok, msg = util.close(got, z['out_' + k], 1.0, rtol=1e-12)
        assert ok, '%s: %s' % (k, msg)
