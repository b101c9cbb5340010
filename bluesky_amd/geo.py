"""Drop-in ``geo.qdrdist_matrix`` / ``geo.kwikqdrdist_matrix`` on MI355X.

Same contract as ``bluesky/tools/geo.py:110-162`` and ``geo.py:347-363`` for
the two ways the reference's callers use them:

* row vectors (``1 x m`` and ``1 x n`` ``np.matrix``, ``traffic/metric.py:596,
  711,1188``): the ``m x n`` outer matrices, returned as ``np.matrix``;
* 1-D arrays (``traffic/asas/SSD.py:169``): the reference's products are then
  all element-wise, so it returns one entry per pair -- ``qdrdist_matrix`` as
  a ``1 x P`` ``np.matrix`` (its ``np.mat`` calls, ``geo.py:141-142``),
  ``kwikqdrdist_matrix`` as ``(P,)`` arrays.

qdr in degrees (KWIK: in [0, 360)); dist in nm (KWIK: metres, as the
reference computes it despite its docstring).  Shapes the reference would
broadcast to a different result (outer qdrdist with m != n and m != 1, outer
KWIK with m != n) raise ``ValueError``.  All compute runs in ``libbsaccel.so``
(``bsa_qdrdist``); there is no CPU fallback.
"""
import numpy as np

from . import _lib


def _mode(args):
    """'outer' for row vectors (1 x k, np.matrix or 2-D), 'pairwise' for 1-D."""
    nd = {np.ndim(a) for a in args}
    if nd == {1}:
        return 'pairwise'
    if nd == {2} and all(np.shape(a)[0] == 1 for a in args):
        return 'outer'
    raise ValueError('expected four 1-D arrays or four 1 x k row vectors, got shapes %s'
                     % [np.shape(a) for a in args])


def _pairwise_operands(lat1, lon1, lat2, lon2):
    """numpy's 1-D broadcasting (a length-1 operand repeats) made explicit."""
    a = [np.asarray(x, dtype=np.float64) for x in (lat1, lon1, lat2, lon2)]
    try:
        b = np.broadcast_arrays(*a)
    except ValueError:
        raise ValueError('1-D operands of lengths %s do not broadcast' % [len(x) for x in a])
    return [np.ascontiguousarray(x) for x in b]


def qdrdist_matrix(lat1, lon1, lat2, lon2, ctx=None):
    """``geo.qdrdist_matrix`` (geo.py:110-162): (qdr [deg], dist [nm])."""
    ctx = ctx or _lib.default_context()
    if _mode((lat1, lon1, lat2, lon2)) == 'pairwise':
        la1, lo1, la2, lo2 = _pairwise_operands(lat1, lon1, lat2, lon2)
        qdr, dist = ctx.qdrdist(la1, lo1, la2, lo2, pairwise=True)
        return np.asmatrix(qdr.reshape(1, -1)), np.asmatrix(dist.reshape(1, -1))
    m, n = np.shape(lat1)[1], np.shape(lat2)[1]
    qdr, dist = ctx.qdrdist(lat1, lon1, lat2, lon2)
    return np.asmatrix(qdr.reshape(m, n)), np.asmatrix(dist.reshape(m, n))


def kwikqdrdist_matrix(lata, lona, latb, lonb, ctx=None):
    """``geo.kwikqdrdist_matrix`` (geo.py:347-363): (qdr [deg, 0..360), dist [m])."""
    ctx = ctx or _lib.default_context()
    if _mode((lata, lona, latb, lonb)) == 'pairwise':
        la, lo, lb, ob = _pairwise_operands(lata, lona, latb, lonb)
        return ctx.qdrdist(la, lo, lb, ob, kwik=True, pairwise=True)
    m, n = np.shape(lata)[1], np.shape(latb)[1]
    qdr, dist = ctx.qdrdist(lata, lona, latb, lonb, kwik=True)
    qdr, dist = qdr.reshape(m, n), dist.reshape(m, n)
    if any(isinstance(a, np.matrix) for a in (lata, lona, latb, lonb)):
        return np.asmatrix(qdr), np.asmatrix(dist)
    return qdr, dist
