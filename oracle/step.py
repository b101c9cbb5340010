"""Oracle composition of the build-defined synthetic sim step.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Order of Traffic.update (bluesky/traffic/traffic.py:383-409) restricted to
the hot path: asas.update (asas.py:473-504: detect, then the resolver only
if confpairs is non-empty -- MVP.resolve, or with ``reso`` off the reference's
default CR DoNothing.resolve) every ``cd_every`` steps with ``asas.active =
inconf``; Pilot.APorASAS (pilot.py:28-63) without wind or with a constant
wind (``p['wind'] = (vnorth, veast)``, windfield.py:150-152) or a 2-D field
(``p['windfield']``, windfield.py:158-179); UpdateAirSpeed /
UpdateGroundSpeed / UpdatePosition (traffic.py:425-483).  With a
``Bookkeeping`` (oracle/asas.py) the CD step instead runs ASAS.update's
resopairs bookkeeping and ResumeNav (asas.py:409-504) and takes asas.active
from it.  ``p['perf']`` (dict actypes, lifttype, limits_fixwing,
limits_rotor) runs OpenAP.update's phase / envelope / acceleration
(oracle/perf.py) before the limits, as Traffic.update does
(traffic.py:397-404).
"""
import numpy as np

from . import kinematics as okin
from . import mvp as omvp
from . import perf as operf
from . import statebased as ocd


def sim_step(st, p, do_cd, bk=None, cd=None):
    """One step on the dict ``st`` (keys of bluesky_amd.resident.initial_state
    plus asas_trk/asas_tas/asas_vs/asas_alt/active).  Returns the new dict.
    ``bk``: an oracle.asas.Bookkeeping, updated in place on CD steps.
    ``cd``: detect results (oracle.statebased.detect_arrays layout) to use
    instead of running the oracle detect -- for sizes where the N^2 oracle
    detect is out of reach and the pair lists were verified separately."""
    st = {k: np.array(v, copy=True) for k, v in st.items()}
    n = len(st['lat'])
    if do_cd:
        traf = dict(lat=st['lat'], lon=st['lon'], trk=st['trk'], gs=st['gs'], alt=st['alt'],
                    vs=st['vs'])
        r = cd if cd is not None else ocd.detect_arrays(traf, traf, p['rpz'], p['hpz'], p['tla'])
        st['n_conf'] = len(r['ci'])
        if not p['reso'] and len(r['ci']):     # CR OFF: DoNothing.resolve (DoNothing.py:11-20)
            st['asas_trk'], st['asas_tas'] = st['ap_trk'].copy(), st['ap_tas'].copy()
            st['asas_vs'], st['asas_alt'] = st['ap_vs'].copy(), st['ap_alt'].copy()
        if p['reso'] and len(r['ci']):         # RESO MVP (asas.py:486-487)
            o = omvp.resolve_arrays(r['ci'], r['cj'], r['qdr'], r['dist'], r['tcpa'],
                                    r['tinconf'], st['gseast'], st['gsnorth'], st['vs'],
                                    st['alt'], st['trk'], st['gs'], st['selalt'], st['ap_vs'],
                                    st['asas_alt'].copy(), p['mvp'])
            st['asas_trk'], st['asas_tas'], st['asas_vs'] = o['trk'], o['tas'], o['vs']
            st['asas_alt'] = o['alt']
        if bk is None:
            st['active'] = np.asarray(r['inconf'], dtype=bool)
        if bk is not None:
            bk.active = np.asarray(st['active'], dtype=bool).copy()
            bk.update(zip(r['ci'], r['cj']), zip(r['li'], r['lj']), st['lat'], st['lon'],
                      st['gseast'], st['gsnorth'], st['trk'], p['rpz'], p['mvp']['Rm'])
            st['active'] = bk.active.copy()
    act = st['active']
    wind = p.get('wind')
    field = p.get('windfield')
    if field is not None:                                     # winddim 2 (windfield.py:158-179)
        vwn, vwe = okin.windfield_2d(st['lat'], st['lon'], field['lat'], field['lon'],
                                     field['vnorth'], field['veast'])
        wind = (vwn, vwe)
    if wind is not None:                                      # pilot.py:31-35
        vwn, vwe = np.ones(n) * wind[0], np.ones(n) * wind[1]
        asastasnorth = st['asas_tas'] * np.cos(np.radians(st['asas_trk'])) - vwn
        asastaseast = st['asas_tas'] * np.sin(np.radians(st['asas_trk'])) - vwe
        asastas = np.sqrt(asastasnorth**2 + asastaseast**2)
    else:
        asastas = st['asas_tas']
    ptrk = np.where(act, st['asas_trk'], st['ap_trk'])
    ptas = np.where(act, asastas, st['ap_tas'])
    palt = np.where(act, st['asas_alt'], st['ap_alt'])
    pvs = np.abs(np.where(act, st['asas_vs'], st['ap_vs']))
    if wind is not None:                                      # pilot.py:51-61
        Vw = np.sqrt(vwn * vwn + vwe * vwe)
        winddir = np.arctan2(vwe, vwn)
        drift = np.radians(ptrk) - winddir
        steer = np.arcsin(np.minimum(1.0, np.maximum(-1.0, Vw * np.sin(drift) /
                                                     np.maximum(0.001, st['tas']))))
        phdg = (ptrk + np.degrees(steer)) % 360.
    else:
        phdg = ptrk % 360.
    env = p.get('limits')
    accel = st['accel']
    pf = p.get('perf')
    if pf is not None:                                        # OpenAP.update (perfoap.py:115-131)
        ph = operf.phase(pf['lifttype'], st['tas'], st['vs'], st['alt'])
        env = operf.envelope(operf.limit_matrix(pf['limits_fixwing'], pf['limits_rotor'], pf['actypes'],
                                                pf['lifttype'], ph))
        accel = operf.acceleration(ph)                        # UpdateAirSpeed (traffic.py:429)
        st['phase'] = ph
    if env is not None:                                       # pilot.py:65-68 (OpenAP)
        ptas, pvs, palt = okin.openap_limits(ptas, pvs, palt, st.get('ax', np.zeros(n)), env)
    s = dict(tas=st['tas'], hdg=st['hdg'], alt=st['alt'], vs=st['vs'], lat=st['lat'], lon=st['lon'],
             ptas=ptas, phdg=phdg, palt=palt, pvs=pvs, bank=st['bank'], eps=st['eps'],
             accel=accel)
    if wind is not None:
        o = okin.step(s, p['simdt'], winddim=1, windnorth=wind[0], windeast=wind[1])
    else:
        o = okin.step(s, p['simdt'])
    for k in ('tas', 'hdg', 'alt', 'vs', 'lat', 'lon', 'gs', 'trk', 'gseast', 'gsnorth', 'ax'):
        st[k] = np.asarray(o[k], dtype=np.float64)
    assert len(st['lat']) == n
    return st
