"""numpy restatement of the standalone ``geo.qdrdist_matrix`` /
``geo.kwikqdrdist_matrix`` producers.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

* outer (row-vector operands, ``traffic/metric.py:596,711,1188``): the
  row-chunked restatements in ``oracle/statebased.py`` (``qdrdist_rows``
  follows ``geo.py:110-162``, ``kwikqdrdist_rows`` ``geo.py:347-363``) over
  all rows.
* pairwise (1-D operands, ``traffic/asas/SSD.py:169``): the same expressions
  with every outer product / transpose of the reference replaced by the
  element-wise product it becomes for 1-D arrays.
Pinned bitwise to the reference by ``tests/golden/geo_*.npz``
(``tools/make_golden.py --geo-only``).
"""
import numpy as np

from .statebased import NM, RE_KWIK, WGS84_A, kwikqdrdist_rows, qdrdist_rows, rwgs84


def qdrdist_outer(lat1, lon1, lat2, lon2):
    """(m x n) qdr [deg], dist [nm]; m == n or m == 1 (geo.py:128)."""
    lat1, lon1, lat2, lon2 = (np.asarray(x, dtype=np.float64).ravel() for x in (lat1, lon1, lat2, lon2))
    assert len(lat1) in (1, len(lat2))
    return qdrdist_rows(lat1, lon1, lat2, lon2, np.arange(len(lat1)))


def kwik_outer(lata, lona, latb, lonb):
    """(n x n) qdr [deg, 0..360), dist [m] (geo.py:351-361)."""
    lata, lona, latb, lonb = (np.asarray(x, dtype=np.float64).ravel() for x in (lata, lona, latb, lonb))
    assert len(lata) == len(latb)
    return kwikqdrdist_rows(lata, lona, latb, lonb, np.arange(len(lata)))


def qdrdist_pairwise(lat1, lon1, lat2, lon2):
    """geo.py:117-160 with 1-D operands: (P,) qdr [deg], dist [nm]."""
    a = WGS84_A
    prodla = lat1 * lat2                                          # geo.py:117
    condition = prodla < 0
    r = np.zeros(prodla.shape)
    r = np.where(condition, r, rwgs84(lat1 + lat2))               # geo.py:121
    num = np.multiply(0.5, (np.multiply(np.abs(lat1), (rwgs84(lat1) + a)) +
                            np.multiply(np.abs(lat2), (rwgs84(lat2) + a))))
    den = np.abs(lat1) + (np.abs(lat2) + (lat1 == 0.) * 0.000001)
    r = np.where(np.invert(condition), r, np.divide(num, den))    # geo.py:125-128
    sin1 = np.radians(lat2 - lat1)
    sin2 = np.radians(lon2 - lon1)
    sinlat1 = np.sin(np.radians(lat1))
    sinlat2 = np.sin(np.radians(lat2))
    coslat1 = np.cos(np.radians(lat1))
    coslat2 = np.cos(np.radians(lat2))
    y = np.multiply(np.sin(sin2), coslat2)
    x = np.multiply(coslat1, sinlat2) - np.multiply(np.multiply(sinlat1, coslat2), np.cos(sin2))
    qdr = np.degrees(np.arctan2(y, x))                            # geo.py:151
    sin10 = np.abs(np.sin(sin1 / 2.))
    sin20 = np.abs(np.sin(sin2 / 2.))
    sqrt = np.multiply(sin10, sin10) + np.multiply(coslat1 * coslat2, np.multiply(sin20, sin20))
    dist_c = np.multiply(2., np.arctan2(np.sqrt(sqrt), np.sqrt(1 - sqrt)))
    return qdr, np.multiply(r / NM, dist_c)                       # geo.py:159


def kwik_pairwise(lata, lona, latb, lonb):
    """geo.py:351-361 with 1-D operands: (P,) qdr [deg, 0..360), dist [m]."""
    dlat = np.radians(latb - lata)
    dlon = np.radians(lonb - lona)
    cavelat = np.cos(np.radians(lata + latb) * 0.5)
    dangle = np.sqrt(np.multiply(dlat, dlat) +
                     np.multiply(np.multiply(dlon, dlon), np.multiply(cavelat, cavelat)))
    return np.degrees(np.arctan2(np.multiply(dlon, cavelat), dlat)) % 360., RE_KWIK * dangle
