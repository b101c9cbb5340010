# Host simulation of the prefilter's culling with the MIDPOINT stage 1 (make_pf_mid):
# stage-1 pair tests (64-row slices x 8-column sub-groups whose boxes may
# interact) for candidate sort orders.  Orders only change the speed, never a
# result.  PYTHONPATH=. python tools/cull_sim2.py box100k
import sys

import numpy as np

from bluesky_amd import synth


def hilbert(X, bits):
    """Skilling's transpose algorithm, n dims of `bits` bits each (n * bits <= 64)."""
    X = X.T.copy().astype(np.int64)
    n = X.shape[0]
    M = 1 << (bits - 1)
    Q = M
    while Q > 1:
        Pm = Q - 1
        for i in range(n):
            m = (X[i] & Q) != 0
            X[0] = np.where(m, X[0] ^ Pm, X[0])
            t = (X[0] ^ X[i]) & Pm
            t = np.where(m, 0, t)
            X[0] ^= t
            X[i] ^= t
        Q >>= 1
    for i in range(1, n):
        X[i] ^= X[i - 1]
    t = np.zeros_like(X[0])
    Q = M
    while Q > 1:
        t = np.where((X[n - 1] & Q) != 0, t ^ (Q - 1), t)
        Q >>= 1
    for i in range(n):
        X[i] ^= t
    key = np.zeros(X.shape[1], dtype=np.uint64)
    for b in range(bits - 1, -1, -1):
        for i in range(n):
            key = (key << np.uint64(1)) | ((X[i] >> b) & 1).astype(np.uint64)
    return key


def quant(v, lo, hi, bits):
    q = ((v - lo) / (hi - lo) * (1 << bits)).astype(np.int64)
    return np.clip(q, 0, (1 << bits) - 1)


def boxes(P, s, lo, hi, g):
    n = (len(P) + g - 1) // g * g
    pad = n - len(P)
    if pad:
        P = np.concatenate([P, np.repeat(P[-1:], pad, 0)])
        s, lo, hi = (np.concatenate([a, np.repeat(a[-1:], pad)]) for a in (s, lo, hi))
    Pg = P.reshape(-1, g, 3)
    return Pg.min(1), Pg.max(1), s.reshape(-1, g).max(1), lo.reshape(-1, g).min(1), hi.reshape(-1, g).max(1)


def count(P, s, lo, hi, gr=64, gc=8):
    rlo, rhi, rs, rvl, rvh = boxes(P, s, lo, hi, gr)
    clo, chi, cs, cvl, cvh = boxes(P, s, lo, hi, gc)
    tot = 0
    for a in range(0, len(rlo), 32):
        gap = np.maximum(0, np.maximum(clo[None] - rhi[a:a + 32, None], rlo[a:a + 32, None] - chi[None]))
        d2 = (gap ** 2).sum(-1)
        st = rs[a:a + 32, None] + cs[None]
        ok = (d2 < st * st) & (cvl[None] < rvh[a:a + 32, None]) & (cvh[None] > rvl[a:a + 32, None])
        tot += ok.sum()
    return tot * gr * gc


def survivors(P, s, lo, hi, sample=2000, seed=1):
    rng = np.random.default_rng(seed)
    rows = rng.choice(len(P), sample, replace=False)
    d2 = ((P[rows, None, :] - P[None, :, :]) ** 2).sum(-1)
    st = s[rows, None] + s[None]
    ok = (d2 < st * st) & (lo[None] < hi[rows, None]) & (hi[None] > lo[rows, None])
    return ok.sum() / sample * len(P)


def main(wl):
    t = synth.workload(wl, seed=7)
    R, H, T = 9260., 304.8, 300.
    lat, lon = np.radians(t.lat), np.radians(t.lon)
    sl, cl, so, co = np.sin(lat), np.cos(lat), np.sin(lon), np.cos(lon)
    u, v = t.gs * np.sin(np.radians(t.trk)), t.gs * np.cos(np.radians(t.trk))
    ht = 0.5 * T
    f = ht / 6371000.0
    P = np.stack([cl * co + f * (-u * so - v * sl * co), cl * so + f * (u * co - v * sl * so), sl + f * (v * cl)], 1)
    ag = np.abs(t.gs) + 0.5e-3
    cmax = (R + (ag + 400.5e-3 + 400) * T) * (1 + 1e-5) / 6.35e6
    kb = np.pi / 2 + (1 + np.pi / 2) / (cl - cmax)
    s = ((0.5 * R + ag * ht) * (1 + 1e-5) + 0.012 * (0.5 * R + ag * T) + ag * ht * kb * cmax) / 6.3e6 \
        + 0.25 * cmax ** 2 + 1e-6
    am = t.alt + t.vs * ht
    h = (0.5 * H + (np.abs(t.vs) + 1.5e-6) * ht) * (1 + 1e-5) + 0.5 + 1e-6 * np.abs(am)
    lo, hi = am - h, am + h
    print('%s stage-1 survivors (sampled) %.3e' % (wl, survivors(P, s, lo, hi)))
    mn, mx = P.min(0), P.max(0)
    span = (mx - mn).max()
    orders = {'hilbert3': hilbert(np.stack([quant(P[:, k], -1, 1, 10) for k in range(3)], 1), 10)}
    climb = (h > 2 * (0.5 * H + 1.0)).astype(np.uint64)
    for ratio in (250., 500., 1000.):
        # altitude scaled so that `ratio` metres of horizontal extent ~ 1 m of altitude
        a_span = span * 6371000.0 / ratio
        q = np.stack([quant(P[:, k], mn[k], mn[k] + span, 16) for k in range(3)] +
                     [quant(am, am.min(), am.min() + a_span, 16)], 1)
        k4 = hilbert(q, 16)
        orders['h4_r%d' % ratio] = k4
        k3 = hilbert(q[:, :3], 16)
        orders['climb|h4_r%d' % ratio] = (climb << np.uint64(63)) | (k4 >> np.uint64(1))
        orders['climb|h3/h4_r%d' % ratio] = np.where(climb == 1, (np.uint64(1) << np.uint64(63)) | (k3 >> np.uint64(1)),
                                                  k4 >> np.uint64(1))
    for name, key in orders.items():
        o = np.argsort(key, kind='stable')
        print('%-22s tests %.3e' % (name, count(P[o], s[o], lo[o], hi[o])))
        sys.stdout.flush()


main(sys.argv[1] if len(sys.argv) > 1 else 'box100k')
