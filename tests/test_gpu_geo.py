"""GPU parity: the standalone geo matrix producers (bsa_qdrdist via
bluesky_amd.geo) against the reference's golden vectors and the oracle.

geo.qdrdist_matrix (geo.py:110-162) and geo.kwikqdrdist_matrix (geo.py:347-363),
outer (row-vector operands, traffic/metric.py:596,711,1188) and pairwise (1-D
operands, traffic/asas/SSD.py:169).  Reals within util.RTOL (1e-9 relative;
ocml's sin/cos/atan2 differ from glibc by <= 1 ulp), NaN where the reference
has NaN (0/0 in the different-hemisphere radius), result type and shape exact.
"""
import numpy as np
import pytest

from bluesky_amd import _lib, geo, synth
from oracle import geo as ogeo
from tests import util

pytestmark = pytest.mark.gpu

GEO = util.golden('geo_*.npz')


def _args(z):
    args = [z[k] for k in ('lat1', 'lon1', 'lat2', 'lon2')]
    if str(z['mode']) == 'outer':
        args = [np.asmatrix(a) for a in args]
    return args


@pytest.mark.parametrize('path', GEO, ids=[util.case_name(p) for p in GEO])
def test_geo_matches_reference_golden(ctx, path):
    z = np.load(path)
    f = geo.qdrdist_matrix if str(z['fn']) == 'qdrdist' else geo.kwikqdrdist_matrix
    qdr, dist = f(*_args(z), ctx=ctx)
    for k, got in (('qdr', qdr), ('dist', dist)):
        assert isinstance(got, np.matrix) == bool(z['is_matrix']), k
        assert tuple(np.shape(got)) == tuple(z['shape']), (k, np.shape(got), z['shape'])
        ok, msg = util.close(np.asarray(got).ravel(), z[k].ravel(), 360.0 if k == 'qdr' else 1e-3)
        assert ok, '%s: %s' % (k, msg)


@pytest.mark.parametrize('n', [1, 63, 64, 257, 2047, 2048, 2049, 2300])
def test_geo_ragged_outer_vs_oracle(ctx, n):
    """Ragged sizes around the 256-lane / 2048-column chunking, both producers."""
    t = synth.global_traffic(n, seed=n)
    u = synth.box(n, 400.0, seed=n + 1, lat0=0.0, lon0=0.0)
    q, d = ctx.qdrdist(t.lat, t.lon, u.lat, u.lon)
    eq, ed = ogeo.qdrdist_outer(t.lat, t.lon, u.lat, u.lon)
    assert util.close(q, eq.ravel(), 360.0)[0] and util.close(d, ed.ravel(), 1e-3)[0]
    q, d = ctx.qdrdist(t.lat, t.lon, u.lat, u.lon, kwik=True)
    eq, ed = ogeo.kwik_outer(t.lat, t.lon, u.lat, u.lon)
    assert util.close(q, eq.ravel(), 360.0)[0] and util.close(d, ed.ravel(), 1.0)[0]


def test_geo_large_outer_rows_and_symmetry(ctx):
    """m = n = 6000 (36 M entries): sampled rows against the oracle, plus the
    size-independent identities of the same-set matrix: dist symmetric and
    zero on the diagonal."""
    t = synth.box(6000, 1500.0, seed=77)
    q, d = ctx.qdrdist(t.lat, t.lon, t.lat, t.lon)
    q, d = q.reshape(6000, 6000), d.reshape(6000, 6000)
    from oracle import statebased as ocd
    rows = np.array([0, 1, 999, 3000, 5999])
    eq, ed = ocd.qdrdist_rows(t.lat, t.lon, t.lat, t.lon, rows)
    assert util.close(q[rows].ravel(), eq.ravel(), 360.0)[0]
    assert util.close(d[rows].ravel(), ed.ravel(), 1e-3)[0]
    assert np.all(np.diag(d) == 0.0)
    assert np.allclose(d, d.T, rtol=1e-12, atol=1e-9)
    assert ctx.geo_last_ms() > 0.0


def test_geo_pairwise_broadcast_and_empty(ctx):
    t = synth.global_traffic(500, seed=5)
    qdr, dist = geo.qdrdist_matrix(t.lat[:1], t.lon[:1], t.lat, t.lon, ctx=ctx)   # (1,) vs (500,)
    eq, ed = ogeo.qdrdist_pairwise(np.repeat(t.lat[:1], 500), np.repeat(t.lon[:1], 500), t.lat, t.lon)
    assert qdr.shape == (1, 500)
    assert util.close(np.asarray(qdr).ravel(), eq, 360.0)[0] and util.close(np.asarray(dist).ravel(), ed, 1e-3)[0]
    q, d = ctx.qdrdist(np.zeros(0), np.zeros(0), np.zeros(0), np.zeros(0), pairwise=True)
    assert q.shape == (0,) and d.shape == (0,)
    q, d = ctx.qdrdist(np.zeros(0), np.zeros(0), np.zeros(0), np.zeros(0))
    assert q.shape == (0,)
    # 1 x 0 against 1 x 500: the reference's (lat1 == 0.)*1e-6 term (geo.py:128)
    # cannot broadcast (1, 500) + (1, 0) and numpy raises; so does the producer
    with pytest.raises(_lib.AccelError, match='m == n or m == 1'):
        ctx.qdrdist(np.zeros(0), np.zeros(0), t.lat, t.lon)


def test_geo_rejects_shapes_the_reference_broadcasts_differently(ctx):
    t = synth.global_traffic(10, seed=1)
    with pytest.raises(_lib.AccelError, match='m == n or m == 1'):
        ctx.qdrdist(t.lat[:3], t.lon[:3], t.lat, t.lon)
    with pytest.raises(_lib.AccelError, match='m == n'):
        ctx.qdrdist(t.lat[:3], t.lon[:3], t.lat, t.lon, kwik=True)
    with pytest.raises(_lib.AccelError, match='equal length'):
        ctx.qdrdist(t.lat[:3], t.lon[:3], t.lat, t.lon, pairwise=True)
    with pytest.raises(ValueError):
        geo.qdrdist_matrix(np.asmatrix(t.lat), t.lon, t.lat, t.lon, ctx=ctx)
