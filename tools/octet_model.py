"""Host model of the prefilter's work at a given cull granularity, in the
DEVICE's own spatial order (3-D Hilbert key of the look-ahead midpoints,
curve_key / k_keys in bsa_cd.hip) and with its own box test
(boxes_may_interact, bsa_box.h): for every (tile pair, 64-row slice) item that
K0d lists, the column sub-groups (8 columns) whose box may interact with the
slice box (the sweep's mask today), and -- finer -- which of the slice's
eight 8-row octets may interact with each such sub-group.

Reports per detect:
  slice x sub-group blocks (the sweep's 64 x 8 stage-1 blocks today),
  octet x sub-group blocks (8 x 8) that survive the finer cull,
  64-lane rounds of an octet sweep: per staged batch of 8 sub-groups,
  ceil(surviving octet blocks / 8) when any octet block can go to any 8-lane
  group ("packed") or max over octets when each octet keeps its 8 lanes
  ("fixed").
Usage: PYTHONPATH=. python tools/octet_model.py [WORKLOAD]"""
import sys

import numpy as np

from bluesky_amd import synth

KT, KG, KS = 512, 64, 8


def expand10(v):
    v = v.astype(np.uint32) & np.uint32(0x3ff)
    v = (v | (v << 16)) & np.uint32(0x030000FF)
    v = (v | (v << 8)) & np.uint32(0x0300F00F)
    v = (v | (v << 4)) & np.uint32(0x030C30C3)
    v = (v | (v << 2)) & np.uint32(0x09249249)
    return v


def curve_key(P):
    """curve_key of bsa_cd.hip: Skilling's transpose, 10 bits per axis."""
    X = [np.clip(((P[:, k] + 1.0) * 512.0).astype(np.int64), 0, 1023).astype(np.uint32) for k in range(3)]
    Q = np.uint32(1 << 9)
    while Q > 1:
        Pm = np.uint32(Q - 1)
        for i in range(3):
            m = (X[i] & Q) != 0
            t = (X[0] ^ X[i]) & Pm
            x0 = np.where(m, X[0] ^ Pm, X[0] ^ t)
            xi = np.where(m, X[i], X[i] ^ t) if i else None
            X[0] = x0
            if i:
                X[i] = xi
        Q = np.uint32(Q >> 1)
    X[1] ^= X[0]
    X[2] ^= X[1]
    t = np.zeros_like(X[0])
    Q = np.uint32(1 << 9)
    while Q > 1:
        t = np.where((X[2] & Q) != 0, t ^ np.uint32(Q - 1), t)
        Q = np.uint32(Q >> 1)
    X = [x ^ t for x in X]
    return (expand10(X[0]) << 2) | (expand10(X[1]) << 1) | expand10(X[2])


def records(t, R=synth.RPZ, H=synth.HPZ, T=synth.TLOOKAHEAD):
    """make_pf_mid (bsa_prep.h) in fp64: midpoint unit vector m, reach s, [lo, hi]."""
    lat, lon = np.radians(t.lat), np.radians(t.lon)
    sl, cl, so, co = np.sin(lat), np.cos(lat), np.sin(lon), np.cos(lon)
    trk = np.radians(t.trk)
    u, v = t.gs * np.sin(trk), t.gs * np.cos(trk)
    ag = np.abs(t.gs) + 0.5e-3
    ht = 0.5 * T
    cmax = (R + (ag + 400.0 + 0.5e-3) * T) * (1 + 1e-5) / 6.35e6
    rhop = cl - cmax
    kb = np.pi / 2 + (1 + np.pi / 2) / rhop
    sm = ((0.5 * R + ag * ht) * (1 + 1e-5) + 0.012 * (0.5 * R + ag * T) + ag * ht * kb * cmax) / 6.3e6 \
        + 0.25 * cmax ** 2 + 1e-6
    f = ht / 6371000.0
    P = np.stack([cl * co + f * (-u * so - v * sl * co), cl * so + f * (u * co - v * sl * so), sl + f * v * cl], 1)
    s = np.where(sm < 0.5, sm, np.inf)
    am = t.alt + t.vs * ht
    h = (0.5 * H + (np.abs(t.vs) + 1.5e-6) * ht) * (1 + 1e-5) + 0.5 + 1e-6 * np.abs(am)
    return P, s, am - h, am + h


def boxes(P, s, lo, hi, g):
    n = (len(P) + g - 1) // g * g
    pad = n - len(P)
    if pad:   # padding records never widen a box
        P = np.concatenate([P, np.repeat(P[-1:], pad, 0)])
        s, lo, hi = (np.concatenate([a, np.repeat(a[-1:], pad)]) for a in (s, lo, hi))
    Pg = P.reshape(-1, g, 3)
    return dict(lo=Pg.min(1), hi=Pg.max(1), s=s.reshape(-1, g).max(1), vlo=lo.reshape(-1, g).min(1),
                vhi=hi.reshape(-1, g).max(1))


def interact(a, ia, b, ib):
    """boxes_may_interact of box a[ia] and b[ib] (broadcast index arrays)."""
    gap = np.maximum(0.0, np.maximum(a['lo'][ia] - b['hi'][ib], b['lo'][ib] - a['hi'][ia]))
    d2 = (gap ** 2).sum(-1)
    st = (a['s'][ia] + b['s'][ib]) * 1.00001 + 1e-5
    return ~(d2 >= st * st) & (b['vlo'][ib] < a['vhi'][ia]) & (b['vhi'][ib] > a['vlo'][ia])


def main(wl):
    t = synth.workload(wl, seed=7)
    P, s, lo, hi = records(t)
    o = np.argsort(curve_key(P), kind='stable')
    P, s, lo, hi = P[o], s[o], lo[o], hi[o]
    n = len(P)
    tb, gb, sb = boxes(P, s, lo, hi, KT), boxes(P, s, lo, hi, KG), boxes(P, s, lo, hi, KS)
    nt = len(tb['s'])
    ti, tj = np.nonzero(interact(tb, np.arange(nt)[:, None], tb, np.arange(nt)[None, :]))
    # items: (tile pair, slice) whose slice (group) box may reach the column tile box
    it_r = (ti[:, None] * 8 + np.arange(8)[None, :]).ravel()
    it_c = np.repeat(tj, 8)
    ok = (it_r < len(gb['s'])) & interact(gb, np.minimum(it_r, len(gb['s']) - 1), tb, it_c)
    it_r, it_c = it_r[ok], it_c[ok]
    print('%s: N=%d, %d tile pairs, %d items' % (wl, n, len(ti), len(it_r)), flush=True)
    nsb = len(sb['s'])
    blocks = rounds_p = rounds_f = blocks8 = batches = 0
    CH = 4096
    for k in range(0, len(it_r), CH):
        r, c = it_r[k:k + CH], it_c[k:k + CH]
        col_sg = c[:, None] * 64 + np.arange(64)[None, :]                   # column sub-groups
        valid = col_sg < nsb
        col_sg = np.minimum(col_sg, nsb - 1)
        gm = valid & interact(gb, r[:, None], sb, col_sg)                   # the sweep's mask
        blocks += int(gm.sum())
        octs = np.minimum(r[:, None] * 8 + np.arange(8)[None, :], nsb - 1)  # the slice's row octets
        om = interact(sb, octs[:, :, None], sb, col_sg[:, None, :]) & gm[:, None, :]   # item x octet x sub-group
        blocks8 += int(om.sum())
        # batches: the mask's set bits in ascending order, 8 at a time
        rank = np.cumsum(gm, 1) - 1
        b_of = np.where(gm, rank // 8, -1)                                  # batch of each sub-group
        nb = (gm.sum(1) + 7) // 8
        batches += int(nb.sum())
        for b in range(int(nb.max()) if len(nb) else 0):
            sel = (b_of == b)[:, None, :] & om                              # octet blocks of batch b
            cnt = sel.sum((1, 2))
            rounds_p += int(((cnt + 7) // 8).sum())
            rounds_f += int(sel.sum(2).max(1).sum())
    print('slice x sub-group blocks (64 x 8): %.4g = %.4g stage-1 tests, %d batches' % (blocks, blocks * 512.0, batches))
    print('octet x sub-group blocks (8 x 8):  %.4g = %.4g stage-1 tests (%.2fx fewer)'
          % (blocks8, blocks8 * 64.0, blocks / max(blocks8, 1) * 8))
    print('64-lane rounds: today %.4g (one per sub-group), octets packed %.4g, octets fixed-lane %.4g'
          % (blocks, rounds_p, rounds_f))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'box100k')
