"""Oracle composition of the build-defined synthetic sim step.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Order of Traffic.update (bluesky/traffic/traffic.py:383-409) restricted to
the hot path: asas.update (asas.py:473-504: detect, then MVP.resolve only if
confpairs is non-empty) every ``cd_every`` steps with ``asas.active =
inconf``; Pilot.APorASAS without wind (pilot.py:28-63); UpdateAirSpeed /
UpdateGroundSpeed / UpdatePosition (traffic.py:425-483).
"""
import numpy as np

from . import kinematics as okin
from . import mvp as omvp
from . import statebased as ocd


def sim_step(st, p, do_cd):
    """One step on the dict ``st`` (keys of bluesky_amd.resident.initial_state
    plus asas_trk/asas_tas/asas_vs/asas_alt/active).  Returns the new dict."""
    st = {k: np.array(v, copy=True) for k, v in st.items()}
    n = len(st['lat'])
    if do_cd:
        traf = dict(lat=st['lat'], lon=st['lon'], trk=st['trk'], gs=st['gs'], alt=st['alt'],
                    vs=st['vs'])
        r = ocd.detect_arrays(traf, traf, p['rpz'], p['hpz'], p['tla'])
        st['n_conf'] = len(r['ci'])
        if p['reso']:
            if len(r['ci']):
                o = omvp.resolve_arrays(r['ci'], r['cj'], r['qdr'], r['dist'], r['tcpa'],
                                        r['tinconf'], st['gseast'], st['gsnorth'], st['vs'],
                                        st['alt'], st['trk'], st['gs'], st['selalt'], st['ap_vs'],
                                        st['asas_alt'].copy(), p['mvp'])
                st['asas_trk'], st['asas_tas'], st['asas_vs'] = o['trk'], o['tas'], o['vs']
                st['asas_alt'] = o['alt']
            st['active'] = np.asarray(r['inconf'], dtype=bool)
    act = st['active']
    ptrk = np.where(act, st['asas_trk'], st['ap_trk'])
    ptas = np.where(act, st['asas_tas'], st['ap_tas'])
    palt = np.where(act, st['asas_alt'], st['ap_alt'])
    pvs = np.abs(np.where(act, st['asas_vs'], st['ap_vs']))
    phdg = ptrk % 360.
    s = dict(tas=st['tas'], hdg=st['hdg'], alt=st['alt'], vs=st['vs'], lat=st['lat'], lon=st['lon'],
             ptas=ptas, phdg=phdg, palt=palt, pvs=pvs, bank=st['bank'], eps=st['eps'],
             accel=st['accel'])
    o = okin.step(s, p['simdt'])
    for k in ('tas', 'hdg', 'alt', 'vs', 'lat', 'lon', 'gs', 'trk', 'gseast', 'gsnorth'):
        st[k] = np.asarray(o[k], dtype=np.float64)
    assert len(st['lat']) == n
    return st
