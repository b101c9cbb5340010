"""numpy restatement of BlueSky's kinematic integration (one sim step).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Follows, in evaluation order:

* ``Traffic.UpdateAirSpeed``    bluesky/traffic/traffic.py:425-454
* ``Traffic.UpdateGroundSpeed`` bluesky/traffic/traffic.py:456-476
  (winddim 0 = no wind, winddim 1 = constant wind; windfield.py:146-152)
* ``Traffic.UpdatePosition``    bluesky/traffic/traffic.py:478-483
* ISA helpers ``vatmos``/``vtemp``/``vvsound``/``vtas2mach``/``vtas2cas``
  bluesky/tools/aero.py:62-104,139-147
"""
import numpy as np

kts = 0.514444              # aero.py:11
ft = 0.3048                 # aero.py:12
fpm = ft / 60.              # aero.py:13
g0 = 9.80665                # aero.py:18
R = 287.05287               # aero.py:19
p0 = 101325.                # aero.py:20
rho0 = 1.225                # aero.py:21
Tstrat = 216.65             # aero.py:23
gamma = 1.40                # aero.py:24
Rearth = 6371000.           # aero.py:28


def vtemp(h):
    return np.maximum(288.15 - 0.0065 * h, Tstrat)


def vatmos(h):
    T = vtemp(h)
    rhotrop = 1.225 * (T / 288.15) ** 4.256848030018761
    dhstrat = np.maximum(0., h - 11000.)
    rho = rhotrop * np.exp(-dhstrat / 6341.552161)
    p = rho * R * T
    return p, rho, T


def vvsound(h):
    T = vtemp(h)
    return np.sqrt(gamma * R * T)


def vtas2mach(tas, h):
    a = vvsound(h)
    return tas / a


def vtas2cas(tas, h):
    p, rho, T = vatmos(h)
    qdyn = p * ((1. + rho * tas * tas / (7. * p)) ** 3.5 - 1.)
    cas = np.sqrt(7. * p0 / rho0 * ((qdyn / p0 + 1.) ** (2. / 7.) - 1.))
    cas = np.where(tas < 0, -1 * cas, cas)
    return cas


def update_airspeed(s, simdt):
    """traffic.py:425-454.  ``s`` holds tas, hdg, alt, vs, bank, eps, accel and
    the pilot targets ptas, phdg, palt, pvs.  Returns a dict of new values."""
    o = {}
    delta_spd = s['ptas'] - s['tas']
    need_ax = np.abs(delta_spd) > kts
    o['ax'] = need_ax * np.sign(delta_spd) * s['accel']
    o['delspd'] = delta_spd
    o['tas'] = s['tas'] + o['ax'] * simdt
    o['cas'] = vtas2cas(o['tas'], s['alt'])
    o['M'] = vtas2mach(o['tas'], s['alt'])

    turnrate = np.degrees(g0 * np.tan(s['bank']) / np.maximum(o['tas'], s['eps']))
    delhdg = (s['phdg'] - s['hdg'] + 180) % 360 - 180
    o['swhdgsel'] = np.abs(delhdg) > np.abs(2 * simdt * turnrate)
    o['hdg'] = (s['hdg'] + simdt * turnrate * o['swhdgsel'] * np.sign(delhdg)) % 360.

    delta_alt = s['palt'] - s['alt']
    o['swaltsel'] = np.abs(delta_alt) > np.maximum(10 * ft, np.abs(2 * simdt * np.abs(s['vs'])))
    target_vs = o['swaltsel'] * np.sign(delta_alt) * np.abs(s['pvs'])
    delta_vs = target_vs - s['vs']
    need_az = np.abs(delta_vs) > 300 * fpm
    o['az'] = need_az * np.sign(delta_vs) * (300 * fpm)
    vs = np.where(need_az, s['vs'] + o['az'] * simdt, target_vs)
    o['vs'] = np.where(np.isfinite(vs), vs, 0)
    return o


def vcas2tas(cas, h):
    """aero.py:128-136."""
    p, rho, T = vatmos(h)
    qdyn = p0 * ((1. + rho0 * cas * cas / (7. * p0)) ** 3.5 - 1.)
    tas = np.sqrt(7. * p / rho * ((1. + qdyn / p) ** (2. / 7.) - 1.))
    return np.where(cas < 0, -1 * tas, tas)


def openap_limits(intent_v_tas, intent_vs, intent_h, ax, env):
    """OpenAP.limits (performance/openap/perfoap.py:185-209), applied by
    Pilot.applylimits (pilot.py:65-68) to the pilot's tas / vs / alt.
    env: per-aircraft envelope dict(hmax, vmin, vmax, vsmin, vsmax, axmax)
    (vmin / vmax are CAS); ax: traf.ax of the previous step."""
    allow_h = np.where(intent_h > env['hmax'], env['hmax'], intent_h)
    intent_v_cas = vtas2cas(intent_v_tas, allow_h)
    allow_v_cas = np.where(intent_v_cas < env['vmin'], env['vmin'], intent_v_cas)
    allow_v_cas = np.where(intent_v_cas > env['vmax'], env['vmax'], allow_v_cas)
    allow_v_tas = vcas2tas(allow_v_cas, allow_h)
    vs_max_with_acc = (1 - ax / env['axmax']) * env['vsmax']
    allow_vs = np.where(intent_vs > env['vsmax'], vs_max_with_acc, intent_vs)
    allow_vs = np.where(intent_vs < env['vsmin'], env['vsmin'], allow_vs)
    return allow_v_tas, allow_vs, allow_h


def windfield_2d(lat, lon, wlat, wlon, wvnorth, wveast):
    """Windfield.getdata for a 2-D field (winddim 2, windfield.py:158-179):
    inverse-distance-squared weights in a flat frame of 1-degree units.
    wlat/wlon: the nvec definition points, wvnorth/wveast their wind [m/s]
    (Windfield.vnorth[0, :] / veast[0, :]).  Same numpy expressions (incl. the
    two matrix products) as the reference, so it is bitwise equal there."""
    eps = 1e-20
    npos = len(lat)
    nvec = len(wlat)
    lat = np.array(lat).reshape((1, npos))
    lon = np.array(lon).reshape((1, npos))
    wl = np.array([np.asarray(wlat, dtype=np.float64)]).transpose()
    wo = np.array([np.asarray(wlon, dtype=np.float64)]).transpose()
    cavelat = np.cos(np.radians(0.5 * (lat + wl)))
    dy = lat - wl
    dx = cavelat * (lon - wo)
    invd2 = 1. / (eps + dx * dx + dy * dy)
    sumsid2 = np.ones((1, nvec)).dot(invd2)
    totals = np.repeat(sumsid2, nvec, axis=0)
    horfact = invd2 / totals
    vnorth = np.asarray(wvnorth, dtype=np.float64).dot(horfact)
    veast = np.asarray(wveast, dtype=np.float64).dot(horfact)
    return vnorth, veast


def update_groundspeed(tas, hdg, alt, winddim=0, windnorth=0.0, windeast=0.0):
    """traffic.py:456-476; windnorth/windeast: scalars (winddim 1) or
    per-aircraft arrays from windfield_2d (winddim 2)."""
    o = {}
    if winddim == 0:
        o['gsnorth'] = tas * np.cos(np.radians(hdg))
        o['gseast'] = tas * np.sin(np.radians(hdg))
        o['gs'] = tas
        o['trk'] = hdg
    else:
        n = len(tas)
        applywind = alt > 50. * ft
        vn = np.ones(n) * windnorth          # windfield.py:150-152
        ve = np.ones(n) * windeast
        o['gsnorth'] = tas * np.cos(np.radians(hdg)) + vn * applywind
        o['gseast'] = tas * np.sin(np.radians(hdg)) + ve * applywind
        o['gs'] = np.logical_not(applywind) * tas + \
            applywind * np.sqrt(o['gsnorth'] ** 2 + o['gseast'] ** 2)
        o['trk'] = np.logical_not(applywind) * hdg + \
            applywind * np.degrees(np.arctan2(o['gseast'], o['gsnorth'])) % 360.
    return o


def update_position(lat, lon, alt, vs, swaltsel, palt, gsnorth, gseast, simdt):
    """traffic.py:478-483."""
    o = {}
    o['alt'] = np.where(swaltsel, alt + vs * simdt, palt)
    o['lat'] = lat + np.degrees(simdt * gsnorth / Rearth)
    o['coslat'] = np.cos(np.deg2rad(o['lat']))
    o['lon'] = lon + np.degrees(simdt * gseast / o['coslat'] / Rearth)
    return o


def step(s, simdt, winddim=0, windnorth=0.0, windeast=0.0):
    """UpdateAirSpeed -> UpdateGroundSpeed -> UpdatePosition (traffic.py:407-409)."""
    o = update_airspeed(s, simdt)
    o.update(update_groundspeed(o['tas'], o['hdg'], s['alt'], winddim, windnorth, windeast))
    o.update(update_position(s['lat'], s['lon'], s['alt'], o['vs'], o['swaltsel'], s['palt'],
                             o['gsnorth'], o['gseast'], simdt))
    return o
