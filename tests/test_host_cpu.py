"""CPU: host-side drop-in plumbing that needs no GPU."""
import types

import numpy as np
import pytest

import bluesky_amd
from bluesky_amd import _lib, kinematics, mvp, resident, statebased, synth


def test_register_uses_asas_plugin_api():
    calls = {'cd': [], 'cr': []}

    class FakeASAS:
        @classmethod
        def addCDMethod(cls, name, module):
            calls['cd'].append((name, module))

        @classmethod
        def addCRMethod(cls, name, module):
            calls['cr'].append((name, module))

    bluesky_amd.register(FakeASAS)
    assert calls['cd'] == [('GPU', statebased), ('GPUKWIK', bluesky_amd.kwik)]
    assert calls['cr'] == [('GPUMVP', mvp)]
    assert callable(bluesky_amd.kwik.detect)
    assert callable(statebased.detect) and callable(mvp.resolve) and callable(mvp.start)


def test_pairs_from_indices():
    ids = ['A', 'B', 'C']
    assert statebased.pairs_from_indices(ids, np.array([0, 2]), np.array([1, 0])) == [('A', 'B'), ('C', 'A')]
    assert statebased.pairs_from_indices(ids, np.array([], int), np.array([], int)) == []


def test_mvp_params_from_asas():
    asas = types.SimpleNamespace(Rm=1.05 * 9260, dhm=1.05 * 304.8, dtlookahead=300.0, vmin=100.0,
                                 vmax=250.0, vsmin=-15.0, vsmax=15.0, swresohoriz=True,
                                 swresospd=False, swresohdg=True, swresovert=False, swprio=True,
                                 priocode='LAY2', swnoreso=False, swresooff=True)
    p = mvp.params_from_asas(asas)
    assert p.priocode == 5 and p.swresohdg == 1 and p.swresooff == 1 and p.Rm == asas.Rm


def test_resident_initial_state_matches_traffic_create():
    t = synth.box(100, 50.0, seed=3)
    s = resident.initial_state(t)
    assert set(_lib.SIM_STATE_FIELDS) <= set(s)
    assert np.allclose(s['ap_vs'], 1500 * 0.3048 / 60.)
    assert np.array_equal(s['tas'], t.gs) and np.array_equal(s['hdg'], t.trk)


def test_kinematics_rejects_3d_wind_fields():
    """winddim 3 fails like the reference's getdata for array positions (windfield.py:177)."""
    traf = types.SimpleNamespace(wind=types.SimpleNamespace(winddim=3))
    with pytest.raises(ValueError, match='windfield.py:177'):
        kinematics.step(traf, 0.05, ctx=types.SimpleNamespace())


def test_kinematics_uploads_2d_wind_field():
    """winddim 2 hands Windfield.lat / lon / vnorth[0, :] / veast[0, :] to the library."""
    got = {}

    class FakeCtx:
        def set_windfield(self, lat, lon, vn, ve):
            got.update(lat=lat, lon=lon, vn=vn, ve=ve)

        def kinematics(self, *a, **k):
            raise _lib.AccelUnavailable('stop here')

    w = types.SimpleNamespace(winddim=2, lat=np.array([1.0, 2.0]), lon=np.array([3.0, 4.0]),
                              vnorth=np.array([[5.0, 6.0], [0.0, 0.0]]), veast=np.array([[7.0, 8.0], [0.0, 0.0]]))
    traf = types.SimpleNamespace(wind=w)
    for k in ('tas', 'hdg', 'alt', 'vs', 'lat', 'lon', 'bank', 'eps'):
        setattr(traf, k, np.zeros(2))
    traf.pilot = types.SimpleNamespace(tas=np.zeros(2), hdg=np.zeros(2), alt=np.zeros(2), vs=np.zeros(2))
    traf.perf = types.SimpleNamespace(acceleration=lambda: np.zeros(2))
    with pytest.raises(_lib.AccelUnavailable):
        kinematics.step(traf, 0.05, ctx=FakeCtx())
    assert np.array_equal(got['vn'], [5.0, 6.0]) and np.array_equal(got['ve'], [7.0, 8.0])


def test_workloads():
    t = synth.workload('box100k', n=2000)
    assert t.ntraf == 2000 and len(t.id) == 2000
    g = synth.global_traffic(5000, seed=1)
    assert np.all(np.abs(g.lat) <= 70.5)


class _GeoCtx:
    """Records what bluesky_amd.geo hands to Context.qdrdist (no GPU needed)."""

    def __init__(self):
        self.calls = []

    def qdrdist(self, lat1, lon1, lat2, lon2, kwik=False, pairwise=False):
        la1, la2 = np.ravel(lat1), np.ravel(lat2)
        self.calls.append((len(la1), len(la2), kwik, pairwise))
        total = len(la1) if pairwise else len(la1) * len(la2)
        return np.arange(total, dtype=np.float64), -np.arange(total, dtype=np.float64)


def test_geo_operand_forms_and_result_types():
    """bluesky_amd.geo mirrors geo.py's result types for the two operand forms
    its callers use (metric.py row vectors, SSD.py 1-D arrays)."""
    from bluesky_amd import geo
    ctx = _GeoCtx()
    a, b = np.linspace(0, 1, 3), np.linspace(0, 1, 4)
    q, d = geo.qdrdist_matrix(np.asmatrix(a), np.asmatrix(a), np.asmatrix(b), np.asmatrix(b), ctx=ctx)
    assert isinstance(q, np.matrix) and q.shape == (3, 4) and q[1, 0] == 4.0
    q, d = geo.qdrdist_matrix(a, a, a, a, ctx=ctx)
    assert isinstance(q, np.matrix) and q.shape == (1, 3)
    q, d = geo.kwikqdrdist_matrix(a, a, a, a, ctx=ctx)
    assert not isinstance(q, np.matrix) and q.shape == (3,)
    q, d = geo.kwikqdrdist_matrix(a[None, :], a[None, :], a[None, :], a[None, :], ctx=ctx)
    assert not isinstance(q, np.matrix) and q.shape == (3, 3)
    q, d = geo.kwikqdrdist_matrix(np.asmatrix(a), np.asmatrix(a), np.asmatrix(a), np.asmatrix(a), ctx=ctx)
    assert isinstance(q, np.matrix)
    # a length-1 1-D operand broadcasts (numpy semantics), made explicit for the C ABI
    geo.qdrdist_matrix(a[:1], a[:1], b, b, ctx=ctx)
    assert ctx.calls[-1] == (4, 4, False, True)
    with pytest.raises(ValueError):
        geo.qdrdist_matrix(a, a, b, b, ctx=ctx)          # 3 vs 4 do not broadcast
    with pytest.raises(ValueError):
        geo.qdrdist_matrix(np.asmatrix(a), a, a, a, ctx=ctx)
    with pytest.raises(ValueError):
        geo.qdrdist_matrix(np.ones((2, 3)), np.ones((2, 3)), np.ones((2, 3)), np.ones((2, 3)), ctx=ctx)


def test_fmod360_reciprocal_quotient_is_exact():
    """bsa_geo_math.h fmod360: q = trunc(|a| * (1/360)), then one neighbour
    tried, gives fmod(a, 360) bitwise (the device function's arithmetic,
    restated in numpy fp64: every operation is IEEE, no contraction) on 2e6
    values: random magnitudes up to 360 * 2^30, the multiples of 360 and their
    ulp neighbours, the range bounds."""
    rng = np.random.default_rng(3)
    a = np.concatenate([rng.uniform(-1, 1, 10 ** 6) * 10 ** rng.uniform(2.5, 11.5, 10 ** 6),
                        rng.uniform(-720, 720, 10 ** 5)])
    k = rng.integers(1, 2 ** 30, 3 * 10 ** 5).astype(np.float64) * 360.0
    a = np.concatenate([a, k, np.nextafter(k, 0), np.nextafter(k, np.inf), -k, [360.0, 720.0, 359.99999999999994,
                                                                                 360 * 2.0 ** 30 - 1]])
    aa = np.abs(a)
    m = (aa >= 360.0) & (aa < 386547056640.0)
    aa = aa[m]
    q = np.trunc(aa * (1.0 / 360.0))
    r = aa - q * 360.0
    lo, hi = r < 0.0, r >= 360.0
    q = np.where(lo, q - 1.0, np.where(hi, q + 1.0, q))
    r = aa - q * 360.0
    got = np.copysign(r, a[m])
    exp = np.fmod(a[m], 360.0)
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))
