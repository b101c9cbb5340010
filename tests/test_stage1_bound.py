"""Host check of the midpoint stage-1 bound (bsa_cd.hip
make_pf_mid): every conflict and LoS pair the reference reports must satisfy
|m_i - m_j| < s_i + s_j and |a_i - a_j| < h_i + h_j with the per-aircraft
midpoint records.  The GPU path tests the same pairs in a projection (which
only shortens the distance) with fp32 rounding covered by the records'
margins; this test checks the derivation itself in fp64, on the golden
fixtures (captured from the reference) and on oracle-evaluated stress sets
(high latitude, fast traffic, long look-ahead, own != intruder)."""
import numpy as np
import pytest

from bluesky_amd import synth
from oracle import statebased as ocd
from tests.util import golden, load_cd, case_name

KVCAP = 400.0
D2R = np.pi / 180.0


def mid_records(lat, lon, trk, gs, alt, vs, rpz, hpz, tla):
    """numpy restatement of make_pf_mid (fp64): m (n, 3), s, a, h."""
    tlap = max(tla, 0.0)
    la, lo = lat * D2R, lon * D2R
    sinl, cosl, sinlo, coslo = np.sin(la), np.cos(la), np.sin(lo), np.cos(lo)
    p = np.stack([cosl * coslo, cosl * sinlo, sinl], axis=1)
    u, v = gs * np.sin(trk * D2R), gs * np.cos(trk * D2R)
    ag = np.abs(gs) + 0.5e-3
    ht = 0.5 * tlap
    cmax = (rpz + (ag + KVCAP + 0.5e-3) * tlap) * (1.0 + 1e-5) / 6.35e6
    rhop = cosl - cmax
    ok = (np.abs(gs) <= KVCAP) & np.isfinite(u) & np.isfinite(v) & (rhop >= 0.05) & (cmax <= 0.1)
    kb = 1.5707963267948966 + 2.5707963267948966 / np.where(ok, rhop, 1.0)
    s = (((0.5 * rpz + ag * ht) * (1.0 + 1e-5) + 0.012 * (0.5 * rpz + ag * tlap) + ag * ht * kb * cmax) / 6.3e6
         + 0.25 * cmax * cmax + 1e-6)
    s = np.where(ok & (s < 0.5), s, np.inf)
    f = ht / 6371000.0
    m = p + f * np.stack([-u * sinlo - v * sinl * coslo, u * coslo - v * sinl * sinlo, v * cosl], axis=1)
    m = np.where(ok[:, None], m, p)
    a = alt + vs * ht
    h = (0.5 * hpz + (np.abs(vs) + 1.5e-6) * ht) * (1.0 + 1e-5) + 0.5 + 1e-6 * np.abs(a)
    return m, s, a, h


def t0_reach(gs, rpz, tla):
    return ((0.5 * rpz + (np.abs(gs) + 0.5e-3) * max(tla, 0.0)) * (1.0 + 1e-5)) / 6.3e6 + 1e-6


def t0_vreach(vs, alt, hpz, tla):
    return (0.5 * hpz + (np.abs(vs) + 0.5e-6) * max(tla, 0.0)) * (1.0 + 1e-5) + 0.5 + 1e-6 * np.abs(alt)


def check_pairs(own, intr, rpz, hpz, tla, pairs):
    """Assert the bound for every (i, j) in pairs; returns (kept_mid, kept_t0) fractions of all pairs."""
    # rows: own[i] position, intruder[i] velocity / altitude; columns: intruder[j]
    # position, own[j] velocity / altitude (StateBasedCD.py:30-40,65-69)
    mr, sr, ar, hr = mid_records(own.lat, own.lon, intr.trk, intr.gs, intr.alt, intr.vs, rpz, hpz, tla)
    mc, sc, ac, hc = mid_records(intr.lat, intr.lon, own.trk, own.gs, own.alt, own.vs, rpz, hpz, tla)
    for (i, j) in pairs:
        i, j = np.asarray(i, dtype=np.int64), np.asarray(j, dtype=np.int64)
        if len(i) == 0:
            continue
        d = np.linalg.norm(mr[i] - mc[j], axis=1)
        hor = d < sr[i] + sc[j]
        ver = np.abs(ac[j] - ar[i]) < hr[i] + hc[j]
        bad = np.flatnonzero(~(hor & ver))
        assert len(bad) == 0, 'pair (%d, %d) dropped: |dm| %.6g vs %.6g, |da| %.6g vs %.6g' % (
            i[bad[0]], j[bad[0]], d[bad[0]], sr[i[bad[0]]] + sc[j[bad[0]]],
            abs(ac[j[bad[0]]] - ar[i[bad[0]]]), hr[i[bad[0]]] + hc[j[bad[0]]])
    # culling statistics on a row sample (the point of the exercise)
    rows = np.arange(0, own.ntraf, max(1, own.ntraf // 200))
    d = np.linalg.norm(mr[rows, None, :] - mc[None, :, :], axis=2)
    kept_mid = ((d < sr[rows, None] + sc[None, :]) &
                (np.abs(ac[None, :] - ar[rows, None]) < hr[rows, None] + hc[None, :])).mean()
    pr = np.stack([np.cos(own.lat * D2R) * np.cos(own.lon * D2R), np.cos(own.lat * D2R) * np.sin(own.lon * D2R),
                   np.sin(own.lat * D2R)], axis=1)
    pc = np.stack([np.cos(intr.lat * D2R) * np.cos(intr.lon * D2R), np.cos(intr.lat * D2R) * np.sin(intr.lon * D2R),
                   np.sin(intr.lat * D2R)], axis=1)
    d0 = np.linalg.norm(pr[rows, None, :] - pc[None, :, :], axis=2)
    s0r, s0c = t0_reach(intr.gs, rpz, tla), t0_reach(own.gs, rpz, tla)
    h0r, h0c = t0_vreach(intr.vs, intr.alt, hpz, tla), t0_vreach(own.vs, own.alt, hpz, tla)
    kept_t0 = ((d0 < s0r[rows, None] + s0c[None, :]) &
               (np.abs(own.alt[None, :] - intr.alt[rows, None]) < h0r[rows, None] + h0c[None, :])).mean()
    return kept_mid, kept_t0


@pytest.mark.parametrize('path', golden('cd_*.npz'), ids=case_name)
def test_midpoint_bound_on_golden(path):
    own, intr, z = load_cd(path)
    check_pairs(own, intr, float(z['rpz']), float(z['hpz']), float(z['tla']),
                [(z['ci'], z['cj']), (z['li'], z['lj'])])


def _stress_sets():
    rng = np.random.default_rng(5)
    out = []
    # dense high-latitude box, fast traffic
    n = 1500
    t = synth.Traffic(66.0 + (rng.random(n) - 0.5) * 6.0, 20.0 + (rng.random(n) - 0.5) * 15.0,
                      rng.uniform(3000, 12000, n), rng.uniform(0, 360, n), rng.uniform(100, 390, n),
                      np.where(rng.random(n) < 0.5, rng.uniform(-15, 15, n), 0.0))
    out.append(('highlat_fast', t, t, 9260.0, 304.8, 300.0))
    # long look-ahead, mid latitude
    t = synth.box(1200, 300.0, seed=9)
    out.append(('box_tla900', t, t, 9260.0, 304.8, 900.0))
    # bigger zone, short look-ahead
    t = synth.box(1200, 150.0, seed=10)
    out.append(('box_rpz20k', t, t, 20000.0, 600.0, 120.0))
    # own != intruder (row velocity from the intruder set)
    a = synth.box(800, 120.0, seed=11)
    b = synth.box(800, 120.0, seed=12)
    out.append(('own_ne_int', a, b, 9260.0, 304.8, 300.0))
    return out


@pytest.mark.parametrize('case', _stress_sets(), ids=lambda c: c[0])
def test_midpoint_bound_on_stress_sets(case):
    name, own, intr, rpz, hpz, tla = case
    exp = ocd.detect_arrays(own, intr, rpz, hpz, tla)
    assert len(exp['ci']) > 0
    kept_mid, kept_t0 = check_pairs(own, intr, rpz, hpz, tla, [(exp['ci'], exp['cj']), (exp['li'], exp['lj'])])
    print('%s: %d conflicts, %d LoS; stage-1 keeps %.4f (midpoint) vs %.4f (t = 0)'
          % (name, len(exp['ci']), len(exp['li']), kept_mid, kept_t0))
