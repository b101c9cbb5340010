# Host simulation of the prefilter's box culling: stage-1 pair tests for a given
# spatial order (Morton / Hilbert) and row-group x column-sub-group size, with
# the same reach bounds and box test as K0/K1a.  PYTHONPATH=. python tools/cull_sim.py box100k
import numpy as np, sys
from bluesky_amd import synth

def expand10(v):
    v = v.astype(np.uint64) & 0x3ff
    v = (v | (v << 16)) & 0x30000ff
    v = (v | (v << 8)) & 0x300f00f
    v = (v | (v << 4)) & 0x30c30c3
    v = (v | (v << 2)) & 0x9249249
    return v

def quant(p):
    return np.clip(((p + 1.0) * 512.0).astype(np.int64), 0, 1023)

def morton(P):
    q = quant(P)
    return (expand10(q[:,0]) << 2) | (expand10(q[:,1]) << 1) | expand10(q[:,2])

def hilbert3(P, bits=10):
    # Skilling's transpose algorithm, vectorised
    X = quant(P).T.copy().astype(np.int64)  # 3 x n
    n = 3
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
        X[i] ^= X[i-1]
    t = np.zeros_like(X[0])
    Q = M
    while Q > 1:
        t = np.where((X[n-1] & Q) != 0, t ^ (Q - 1), t)
        Q >>= 1
    for i in range(n):
        X[i] ^= t
    # interleave transpose -> key (bit b of X[i] -> position)
    key = np.zeros(X.shape[1], dtype=np.uint64)
    for b in range(bits - 1, -1, -1):
        for i in range(n):
            key = (key << np.uint64(1)) | ((X[i] >> b) & 1).astype(np.uint64)
    return key

def boxes(P, s, lo, hi, g):
    n = len(P) // g * g
    Pg = P[:n].reshape(-1, g, 3)
    return (Pg.min(1), Pg.max(1), s[:n].reshape(-1, g).max(1), lo[:n].reshape(-1, g).min(1), hi[:n].reshape(-1, g).max(1))

def count(P, s, lo, hi, gr=64, gc=16):
    rlo, rhi, rs, rvl, rvh = boxes(P, s, lo, hi, gr)
    clo, chi, cs, cvl, cvh = boxes(P, s, lo, hi, gc)
    tot = 0
    for a in range(0, len(rlo), 64):
        gap = np.maximum(0, np.maximum(clo[None] - rhi[a:a+64, None], rlo[a:a+64, None] - chi[None]))
        d2 = (gap**2).sum(-1)
        st = rs[a:a+64, None] + cs[None]
        ok = (d2 < st*st) & (cvl[None] < rvh[a:a+64, None]) & (cvh[None] > rvl[a:a+64, None])
        tot += ok.sum()
    return tot * gr * gc

def main(wl):
    t = synth.workload(wl, seed=7)
    lat, lon = np.radians(t.lat), np.radians(t.lon)
    P = np.stack([np.cos(lat)*np.cos(lon), np.cos(lat)*np.sin(lon), np.sin(lat)], 1)
    R, H, T = 9260., 304.8, 300.
    s = ((0.5*R + (np.abs(t.gs)+0.5e-3)*T)*(1+1e-5))/6.3e6 + 1e-6
    h = (0.5*H + (np.abs(t.vs)+0.5e-6)*T)*(1+1e-5) + 0.5 + 1e-6*np.abs(t.alt)
    lo, hi = t.alt - h, t.alt + h
    for name, key in (('morton', morton(P)), ('hilbert', hilbert3(P))):
        o = np.argsort(key, kind='stable')
        for gr, gc in ((64, 16), (64, 8), (32, 16), (32, 8)):
            print(wl, name, gr, gc, '%.3e' % count(P[o], s[o], lo[o], hi[o], gr, gc))
        sys.stdout.flush()

main(sys.argv[1])
