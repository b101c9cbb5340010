"""Drop-in kinematic integration on MI355X.

Replaces ``Traffic.UpdateAirSpeed`` + ``UpdateGroundSpeed`` +
``UpdatePosition`` (bluesky/traffic/traffic.py:425-483), which
``Traffic.update`` calls back to back (traffic.py:407-409), by ONE fused HIP
kernel.  BlueSky has no plugin API for kinematics, so
``install(traf)`` rebinds the three methods on the instance: the fused step
runs in ``UpdateAirSpeed`` and the other two become no-ops.

Supports winddim 0 (no wind), 1 (constant wind) and 2 (2-D field: the
inverse-distance-squared interpolation of windfield.py:158-179, per aircraft
on the device, bsa_set_windfield).  winddim 3 (altitude profiles) raises
ValueError, as the reference's own getdata does for array positions
(windfield.py:177 compares an ndarray with None in a boolean context).
"""
import types

import numpy as np

from . import _lib

KTS = 0.514444


def step(traf, simdt, ctx=None):
    """One fused UpdateAirSpeed/GroundSpeed/Position on ``traf`` (bs.traf-like)."""
    ctx = ctx or _lib.default_context()
    winddim = int(getattr(traf.wind, 'winddim', 0)) if hasattr(traf, 'wind') else 0
    vn = ve = 0.0
    if winddim == 1:
        vn = float(traf.wind.vnorth[0, 0])   # windfield.py:150-152
        ve = float(traf.wind.veast[0, 0])
    elif winddim == 2:
        w = traf.wind                         # Windfield.lat / lon / vnorth[0, :] / veast[0, :]
        ctx.set_windfield(w.lat, w.lon, np.asarray(w.vnorth)[0, :], np.asarray(w.veast)[0, :])
    elif winddim > 2:
        raise ValueError('winddim %d: the reference\'s 3-D wind interpolation fails for array '
                         'positions (windfield.py:177)' % winddim)
    state = {k: np.array(getattr(traf, k), dtype=np.float64, copy=True)
             for k in ('tas', 'hdg', 'alt', 'vs', 'lat', 'lon')}
    inputs = dict(ptas=traf.pilot.tas, phdg=traf.pilot.hdg, palt=traf.pilot.alt, pvs=traf.pilot.vs,
                  bank=traf.bank, eps=traf.eps, accel=traf.perf.acceleration())
    o = ctx.kinematics(simdt, state, inputs, winddim, vn, ve)
    # traffic.py:428-454
    traf.ax, traf.delspd = o['ax'], o['delspd']
    traf.tas, traf.cas, traf.M = state['tas'], o['cas'], o['mach']
    traf.swhdgsel, traf.hdg = o['swhdgsel'], state['hdg']
    traf.swaltsel, traf.az, traf.vs = o['swaltsel'], o['az'], state['vs']
    # traffic.py:458-476
    traf.gsnorth, traf.gseast, traf.gs, traf.trk = o['gsnorth'], o['gseast'], o['gs'], o['trk']
    # traffic.py:480-483
    traf.alt, traf.lat, traf.coslat, traf.lon = state['alt'], state['lat'], o['coslat'], state['lon']


def install(traf, ctx=None):
    """Rebind the three Update* methods of a Traffic instance to the fused kernel."""
    def _air(self, simdt, simt=None):
        step(self, simdt, ctx)

    def _noop(self, simdt):
        return None

    traf.UpdateAirSpeed = types.MethodType(_air, traf)
    traf.UpdateGroundSpeed = types.MethodType(_noop, traf)
    traf.UpdatePosition = types.MethodType(_noop, traf)
    return traf
