"""Drop-in MVP conflict resolution on MI355X (CR method module).

Same contract as ``bluesky/traffic/asas/MVP.py``: ``start(asas)`` and
``resolve(asas, traf)``; reads ``asas.confpairs/qdr/dist/tcpa/tLOS`` and the
ASAS switches, writes ``asas.trk, tas, vs, alt, asase, asasn, asaseval``
(MVP.py:14-143).  Register with ``bluesky_amd.register()``
(``ASAS.addCRMethod('GPUMVP', ...)``, asas.py:53-55) and select with
``RESO GPUMVP`` (stack.py:631).

When the pairs came from ``bluesky_amd.statebased.detect`` on the same
traffic, the device-resident pairs of that detect are consumed directly;
otherwise (e.g. numpy StateBasedCD) they are uploaded with ``bsa_set_pairs``.
"""
import numpy as np

from . import _lib, statebased

FT = 0.3048


def start(asas):
    """MVP.py:11-12."""
    pass


def params_from_asas(asas):
    """bsa_mvp_params from the ASAS object's scalars (asas.py:81-112)."""
    return _lib.MvpParams(
        Rm=float(asas.Rm), dhm=float(asas.dhm), dtlookahead=float(asas.dtlookahead),
        vmin=float(asas.vmin), vmax=float(asas.vmax), vsmin=float(asas.vsmin),
        vsmax=float(asas.vsmax), swresohoriz=int(bool(asas.swresohoriz)),
        swresospd=int(bool(asas.swresospd)), swresohdg=int(bool(asas.swresohdg)),
        swresovert=int(bool(asas.swresovert)), swprio=int(bool(asas.swprio)),
        priocode=_lib.PRIO_CODES.get(asas.priocode, 0), swnoreso=int(bool(asas.swnoreso)),
        swresooff=int(bool(asas.swresooff)))


def _membership(ids, names):
    if not names:
        return None
    s = set(names)
    return np.fromiter((i in s for i in ids), dtype=np.uint8, count=len(ids))


def resolve(asas, traf, ctx=None):
    """MVP.resolve drop-in (MVP.py:14-143)."""
    if not asas.swasas:
        return
    ctx = ctx or _lib.default_context()
    n = traf.ntraf
    last = statebased.last_detect()
    # the device still holds that detect's pairs only if nothing replaced them since
    # (another detect, set_pairs or set_state on the same context bumps ctx.gen)
    reuse = (last is not None and last['confpairs'] is asas.confpairs and last['ctx'] is ctx
             and last['n'] == n and last['gen'] == ctx.gen)
    if not reuse:
        ctx.set_state(traf.lat, traf.lon, traf.trk, traf.gs, traf.alt, traf.vs)
        idx = {k: i for i, k in enumerate(traf.id)}   # MVP.py:34-35 traf.id.index
        ci = np.fromiter((idx[a] for a, _ in asas.confpairs), dtype=np.int32, count=len(asas.confpairs))
        cj = np.fromiter((idx[b] for _, b in asas.confpairs), dtype=np.int32, count=len(asas.confpairs))
        order = np.argsort(ci, kind='stable')          # per-row fold order is preserved
        ctx.set_pairs(ci[order], cj[order], np.asarray(asas.qdr)[order], np.asarray(asas.dist)[order],
                      np.asarray(asas.tcpa)[order], np.asarray(asas.tLOS)[order])
    noreso = _membership(traf.id, asas.noresolst) if asas.swnoreso else None
    resooff = _membership(traf.id, asas.resoofflst) if asas.swresooff else None
    alt = np.array(asas.alt, dtype=np.float64, copy=True)
    o = ctx.mvp(params_from_asas(asas), traf.gseast, traf.gsnorth, traf.selalt, traf.ap.vs, alt,
                noreso=noreso, resooff=resooff)
    asas.trk = o['trk']
    asas.tas = o['tas']
    asas.vs = o['vs']
    asas.alt = alt
    asas.asase = o['asase']
    asas.asasn = o['asasn']
    if not asas.asaseval:
        asas.asaseval = True
