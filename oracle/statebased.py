"""Row-chunked numpy restatement of BlueSky's StateBased conflict detection.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Follows, expression by expression and in the same evaluation order:

* ``bluesky/tools/geo.py:32-54``   ``rwgs84_matrix``
* ``bluesky/tools/geo.py:110-162`` ``qdrdist_matrix`` -- including the two
  quirks the GPU path must reproduce: the WGS-84 radius is evaluated at the
  SUM of the two latitudes (``geo.py:121``), and the different-hemisphere
  denominator adds ``(lat1 == 0.)*1e-6`` indexed by the COLUMN (``geo.py:125-128``).
* ``bluesky/traffic/asas/StateBasedCD.py:7-103`` ``detect``.  Note the mixed
  orientation (``StateBasedCD.py:39-40,65-69``): geometry row ``i`` is the
  ownship, but ``du[i,j] = own.u[j] - int.u[i]`` and ``dalt[i,j] =
  own.alt[j] - int.alt[i]``.

The ``np.matrix`` outer products of the reference (``lat1.T * lat2`` and
``coslat1.T * coslat2``, k = 1 matmuls) are single rounded products, so
``np.multiply.outer`` gives the same bits.  Rows are processed in chunks so
peak memory is ~30 x 8 x rows x N bytes instead of the reference's
25.5 x 8 x N^2.
"""
import numpy as np

NM = 1852.0                 # bluesky/tools/aero.py:16 (== geo.py:7)
WGS84_A = 6378137.0         # geo.py:38
WGS84_B = 6356752.314245    # geo.py:39


def rwgs84(latd):
    """geo.py:32-54 (elementwise; identical op order to rwgs84_matrix)."""
    a = WGS84_A
    b = WGS84_B
    lat = np.radians(latd)
    coslat = np.cos(lat)
    sinlat = np.sin(lat)
    an = a * a * coslat
    bn = b * b * sinlat
    ad = a * coslat
    bd = b * sinlat
    anan = np.multiply(an, an)
    bnbn = np.multiply(bn, bn)
    adad = np.multiply(ad, ad)
    bdbd = np.multiply(bd, bd)
    return np.sqrt(np.divide(anan + bnbn, adad + bdbd))


def qdrdist_rows(lat1, lon1, lat2, lon2, rows):
    """``geo.qdrdist_matrix`` restricted to the ownship rows ``rows``.

    lat1/lon1: full ownship vectors (N,), lat2/lon2: intruder vectors (M,).
    Returns (qdr [deg], dist [nm]) of shape (len(rows), M).
    """
    a = WGS84_A
    l1 = lat1[rows][:, None]          # lat1.T  (rows x 1)
    o1 = lon1[rows][:, None]
    l2 = lat2[None, :]                # lat2    (1 x M)
    o2 = lon2[None, :]

    prodla = np.multiply.outer(lat1[rows], lat2)            # geo.py:118
    condition = prodla < 0

    r = np.zeros(prodla.shape)
    r = np.where(condition, r, rwgs84(l1 + l2))              # geo.py:122

    # geo.py:126-129 (different hemisphere); (lat1 == 0.) is indexed by column
    num = np.multiply(0.5, (np.multiply(np.abs(l1), (rwgs84(l1) + a)) +
                            np.multiply(np.abs(l2), (rwgs84(l2) + a))))
    den = np.abs(l1) + (np.abs(l2) + (lat1[None, :] == 0.) * 0.000001)
    r = np.where(np.invert(condition), r, np.divide(num, den))

    diff_lat = l2 - l1                                        # geo.py:131
    diff_lon = o2 - o1

    sin1 = np.radians(diff_lat)
    sin2 = np.radians(diff_lon)

    sinlat1 = np.sin(np.radians(l1))
    sinlat2 = np.sin(np.radians(l2))
    coslat1 = np.cos(np.radians(l1))
    coslat2 = np.cos(np.radians(l2))

    sin21 = np.sin(sin2)
    cos21 = np.cos(sin2)
    y = np.multiply(sin21, coslat2)

    x1 = np.multiply(coslat1, sinlat2)
    x2 = np.multiply(sinlat1, coslat2)
    x3 = np.multiply(x2, cos21)
    x = x1 - x3

    qdr = np.degrees(np.arctan2(y, x))                        # geo.py:152

    sin10 = np.abs(np.sin(sin1 / 2.))
    sin20 = np.abs(np.sin(sin2 / 2.))
    sin1sin1 = np.multiply(sin10, sin10)
    sin2sin2 = np.multiply(sin20, sin20)
    cc = np.multiply.outer(coslat1[:, 0], coslat2[0, :])      # coslat1.T * coslat2
    sqrt = sin1sin1 + np.multiply(cc, sin2sin2)
    dist_c = np.multiply(2., np.arctan2(np.sqrt(sqrt), np.sqrt(1 - sqrt)))
    dist = np.multiply(r / NM, dist_c)                        # geo.py:160
    return qdr, dist


RE_KWIK = 6371000.          # geo.py:352


def kwikqdrdist_rows(lata, lona, latb, lonb, rows):
    """``geo.kwikqdrdist_matrix`` (geo.py:347-363) restricted to the rows
    ``rows``; returns (qdr [deg, 0..360), dist [m]).  Note the transposes as
    written: ``dlat[i,j] = latb[j] - lata[i]`` but ``cavelat[i,j]`` uses
    ``lata[j] + latb[i]`` (symmetric only when a == b)."""
    la = lata[rows][:, None]                                  # lata.T
    lo = lona[rows][:, None]
    dlat = np.radians(latb[None, :] - la)                     # geo.py:353
    dlon = np.radians(lonb[None, :] - lo)                     # geo.py:354
    cavelat = np.cos(np.radians(lata[None, :] + latb[rows][:, None]) * 0.5)   # geo.py:355
    dangle = np.sqrt(np.multiply(dlat, dlat) +
                     np.multiply(np.multiply(dlon, dlon), np.multiply(cavelat, cavelat)))
    dist = RE_KWIK * dangle
    qdr = np.degrees(np.arctan2(np.multiply(dlon, cavelat), dlat)) % 360.
    return qdr, dist


def detect_rows(own, intr, RPZ, HPZ, tlookahead, rows, want_dcpa=False, kwik=False):
    """StateBasedCD.detect (StateBasedCD.py:7-103) for the ownship rows ``rows``.

    ``own``/``intr`` are mappings (or objects) with numpy fp64 vectors
    ``lat, lon, trk, gs, alt, vs`` of equal length N.  Returns a dict with the
    per-pair masks' row-major indices and values for these rows.
    """
    g = _getter(own)
    h = _getter(intr)
    n = len(g('lat'))
    rows = np.asarray(rows, dtype=np.int64)
    I = (rows[:, None] == np.arange(n)[None, :]).astype(np.float64)

    if kwik:
        # KWIK variant: kwikqdrdist_matrix swapped in for qdrdist_matrix, its
        # metre distance handed over in nm (bluesky_amd/kwik.py)
        qdr, dist_m = kwikqdrdist_rows(g('lat'), g('lon'), h('lat'), h('lon'), rows)
        dist = dist_m / NM
    else:
        qdr, dist = qdrdist_rows(g('lat'), g('lon'), h('lat'), h('lon'), rows)
    qdr = np.array(qdr)
    dist = np.array(dist) * NM + 1e9 * I                      # StateBasedCD.py:22

    qdrrad = np.radians(qdr)
    dx = dist * np.sin(qdrrad)
    dy = dist * np.cos(qdrrad)

    owntrkrad = np.radians(g('trk'))
    ownu = g('gs') * np.sin(owntrkrad).reshape((1, n))
    ownv = g('gs') * np.cos(owntrkrad).reshape((1, n))
    inttrkrad = np.radians(h('trk'))
    intu = h('gs') * np.sin(inttrkrad).reshape((1, n))
    intv = h('gs') * np.cos(inttrkrad).reshape((1, n))

    du = ownu - intu.T[rows]                                  # StateBasedCD.py:39
    dv = ownv - intv.T[rows]

    dv2 = du * du + dv * dv
    dv2 = np.where(np.abs(dv2) < 1e-6, 1e-6, dv2)
    vrel = np.sqrt(dv2)

    tcpa = -(du * dx + dv * dy) / dv2 + 1e9 * I               # StateBasedCD.py:46

    dcpa2 = dist * dist - tcpa * tcpa * dv2

    R2 = RPZ * RPZ
    swhorconf = dcpa2 < R2

    dxinhor = np.sqrt(np.maximum(0., R2 - dcpa2))
    dtinhor = dxinhor / vrel

    tinhor = np.where(swhorconf, tcpa - dtinhor, 1e8)
    touthor = np.where(swhorconf, tcpa + dtinhor, -1e8)

    dalt = g('alt').reshape((1, n)) - \
        h('alt').reshape((1, n)).T[rows] + 1e9 * I            # StateBasedCD.py:65
    dvs = g('vs').reshape(1, n) - h('vs').reshape(1, n).T[rows]
    dvs = np.where(np.abs(dvs) < 1e-6, 1e-6, dvs)

    tcrosshi = (dalt + HPZ) / -dvs
    tcrosslo = (dalt - HPZ) / -dvs
    tinver = np.minimum(tcrosshi, tcrosslo)
    toutver = np.maximum(tcrosshi, tcrosslo)

    tinconf = np.maximum(tinver, tinhor)
    toutconf = np.minimum(toutver, touthor)

    swconfl = np.array(swhorconf * (tinconf <= toutconf) * (toutconf > 0.0) *
                       (tinconf < tlookahead) * (1.0 - I), dtype=bool)

    inconf = np.any(swconfl, 1)
    tcpamax = np.max(tcpa * swconfl, 1)

    ci, cj = np.where(swconfl)
    swlos = (dist < RPZ) * (np.abs(dalt) < HPZ)
    li, lj = np.where(swlos)

    out = dict(ci=rows[ci], cj=cj.astype(np.int64), li=rows[li],
               lj=lj.astype(np.int64), inconf=inconf, tcpamax=tcpamax,
               qdr=qdr[swconfl], dist=dist[swconfl], tcpa=tcpa[swconfl],
               tinconf=tinconf[swconfl])
    if want_dcpa:
        # build-defined extension: sqrt(max(dcpa2, 0)) [m]
        out['dcpa'] = np.sqrt(np.maximum(dcpa2[swconfl], 0.0))
    return out


def _getter(obj):
    if isinstance(obj, dict):
        return lambda k: np.asarray(obj[k], dtype=np.float64)
    return lambda k: np.asarray(getattr(obj, k), dtype=np.float64)


def chunk_rows(n, budget_bytes=2 << 30):
    """Rows per chunk so that ~32 live (rows x n) fp64 temporaries fit."""
    return int(max(1, min(n, budget_bytes // (32 * 8 * max(n, 1)))))


def detect_arrays(own, intr, RPZ, HPZ, tlookahead, want_dcpa=False,
                  rows=None, budget_bytes=2 << 30, kwik=False):
    """Full (or row-subset) detect as index/value arrays, chunked over rows."""
    n = len(_getter(own)('lat'))
    rows = np.arange(n) if rows is None else np.asarray(rows, dtype=np.int64)
    step = chunk_rows(n, budget_bytes)
    parts = [detect_rows(own, intr, RPZ, HPZ, tlookahead, rows[k:k + step],
                         want_dcpa, kwik) for k in range(0, len(rows), step)]
    if not parts:
        parts = [detect_rows(own, intr, RPZ, HPZ, tlookahead, rows, want_dcpa, kwik)]
    out = {}
    for key in parts[0]:
        out[key] = np.concatenate([p[key] for p in parts])
    return out


def detect(ownship, intruder, RPZ, HPZ, tlookahead):
    """Same contract and return types as StateBasedCD.detect (8-tuple)."""
    r = detect_arrays(ownship, intruder, RPZ, HPZ, tlookahead)
    ids = list(ownship['id'] if isinstance(ownship, dict) else ownship.id)
    confpairs = [(ids[i], ids[j]) for i, j in zip(r['ci'], r['cj'])]
    lospairs = [(ids[i], ids[j]) for i, j in zip(r['li'], r['lj'])]
    return (confpairs, lospairs, r['inconf'], r['tcpamax'], r['qdr'],
            r['dist'], r['tcpa'], r['tinconf'])
