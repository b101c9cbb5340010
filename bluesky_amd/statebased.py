"""Drop-in StateBased conflict detection on MI355X.

Same contract as ``bluesky/traffic/asas/StateBasedCD.py:7-103``::

    confpairs, lospairs, inconf, tcpamax, qdr, dist, tcpa, tinconf = \\
        detect(ownship, intruder, RPZ, HPZ, tlookahead)

* ``ownship``/``intruder``: objects with fp64 ``lat, lon, trk, gs, alt, vs``
  arrays and an ``id`` list (``bs.traf``); ``RPZ``/``HPZ`` in metres,
  ``tlookahead`` in seconds (``asas.py:481-483`` passes ``self.R``,
  ``self.dh``, ``self.dtlookahead``).
* returns the reference's types: lists of ``(id_i, id_j)`` tuples in
  row-major order, ``inconf`` bool ndarray, ``tcpamax`` and the four per-pair
  fp64 arrays in the same order as ``confpairs``.

``detect(..., with_dcpa=True)`` is a build-defined extension returning the
north-star 9-tuple ``(confpairs, lospairs, inconf, tcpamax, qdr, dist, dcpa,
tcpa, tLOS)`` with ``dcpa = sqrt(max(dcpa2, 0))`` [m].

Register it with ``bluesky_amd.register()`` (``ASAS.addCDMethod('GPU', ...)``,
``asas.py:49-51``) and select it with ``CDMETHOD GPU`` (``stack.py:284``).
All compute runs in ``libbsaccel.so``; there is no CPU fallback.
"""
import gc
import time

import numpy as np

from . import _lib


def _upload(ctx, ownship, intruder):
    ctx.set_state(ownship.lat, ownship.lon, ownship.trk, ownship.gs, ownship.alt, ownship.vs)
    if intruder is not ownship:
        ctx.set_intruder(intruder.lat, intruder.lon, intruder.trk, intruder.gs, intruder.alt,
                         intruder.vs)


def detect_indices(ownship, intruder, RPZ, HPZ, tlookahead, with_dcpa=False, ctx=None,
                   row_begin=0, row_end=-1, noprune=False, kwik=False, stage1_t0=False, timings=None):
    """Index-array form: dict(ci, cj, qdr, dist, tcpa, tinconf[, dcpa], li, lj, inconf, tcpamax).
    ``kwik=True``: the opt-in flat-earth variant (``bluesky_amd.kwik``).
    ``noprune`` / ``stage1_t0``: test aids selecting other (result-identical) culling.
    ``timings``: optional dict receiving the wall time [s] of the host-to-device
    upload (``h2d``), the detect up to its completion (``detect``) and the
    device-to-host copy of the results (``d2h``)."""
    ctx = ctx or _lib.default_context()
    t0 = time.perf_counter()
    _upload(ctx, ownship, intruder)
    t1 = time.perf_counter()
    flags = ((_lib.FLAG_WITH_DCPA if with_dcpa else 0) | (_lib.FLAG_NOPRUNE if noprune else 0) |
             (_lib.FLAG_KWIK if kwik else 0) | (_lib.FLAG_STAGE1_T0 if stage1_t0 else 0))
    nc, nl = ctx.detect(RPZ, HPZ, tlookahead, flags, row_begin, row_end)
    t2 = time.perf_counter()
    o = ctx.fetch_pairs(nc, nl, with_dcpa)
    if timings is not None:
        timings.update(h2d=t1 - t0, detect=t2 - t1, d2h=time.perf_counter() - t2)
    return o


def pairs_from_indices(ids, i, j):
    """[(ids[i0], ids[j0]), ...] built vectorised through an object array, with
    the cyclic garbage collector paused: ~10^5 fresh tuples would otherwise
    trigger several collections (1.6x the build time)."""
    if len(i) == 0:
        return []
    a = ids if isinstance(ids, np.ndarray) and ids.dtype == object else np.asarray(ids, dtype=object)
    was = gc.isenabled()
    gc.disable()
    try:
        return list(zip(a[i].tolist(), a[j].tolist()))
    finally:
        if was:
            gc.enable()


_last = {}


def last_detect():
    """The last drop-in detect's confpairs list, context, n and the context's
    generation right after it (for MVP reuse)."""
    return _last or None


def detect(ownship, intruder, RPZ, HPZ, tlookahead, with_dcpa=False, kwik=False, timings=None, ctx=None):
    """StateBasedCD.detect drop-in (8-tuple; 9-tuple with ``with_dcpa=True``).
    ``timings``: optional dict, filled as in ``detect_indices`` plus ``tuples``
    (building the lists of id tuples) and ``total``.  ``ctx``: a Context other
    than the process-wide default one."""
    ctx = ctx or _lib.default_context()
    t0 = time.perf_counter()
    o = detect_indices(ownship, intruder, RPZ, HPZ, tlookahead, with_dcpa=with_dcpa, ctx=ctx,
                       kwik=kwik, timings=timings)
    t1 = time.perf_counter()
    ids = np.asarray(ownship.id, dtype=object)
    confpairs = pairs_from_indices(ids, o['ci'], o['cj'])
    lospairs = pairs_from_indices(ids, o['li'], o['lj'])
    if timings is not None:
        t2 = time.perf_counter()
        timings.update(tuples=t2 - t1, total=t2 - t0)
    _last.clear()
    if intruder is ownship:
        _last.update(confpairs=confpairs, ctx=ctx, n=len(ids), gen=ctx.gen)
    inconf = o['inconf'].astype(bool)
    if with_dcpa:
        return (confpairs, lospairs, inconf, o['tcpamax'], o['qdr'], o['dist'], o['dcpa'],
                o['tcpa'], o['tinconf'])
    return confpairs, lospairs, inconf, o['tcpamax'], o['qdr'], o['dist'], o['tcpa'], o['tinconf']


class ConflictDetection:
    """Object form named in the north-star contract:
    ``ConflictDetection().detect(ownship, intruder, rpz, hpz, dtlookahead)``."""

    def __init__(self, device=0, with_dcpa=False):
        self.device = device
        self.with_dcpa = with_dcpa

    def detect(self, ownship, intruder, rpz, hpz, dtlookahead):
        ctx = _lib.default_context(self.device)
        o = detect_indices(ownship, intruder, rpz, hpz, dtlookahead, self.with_dcpa, ctx=ctx)
        ids = np.asarray(ownship.id, dtype=object)
        res = [pairs_from_indices(ids, o['ci'], o['cj']), pairs_from_indices(ids, o['li'], o['lj']),
               o['inconf'].astype(bool), o['tcpamax'], o['qdr'], o['dist']]
        if self.with_dcpa:
            res.append(o['dcpa'])
        res += [o['tcpa'], o['tinconf']]
        return tuple(res)
