"""numpy restatement of BlueSky's MVP conflict resolution.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Follows ``bluesky/traffic/asas/MVP.py``:

* ``resolve``   MVP.py:14-143 -- the pair loop (33-61) is a sequential fold
  of ``dv[id1] -= dv_mvp`` in confpair order; only ``dv[id1]`` is ever written
  (the ``dv2`` returned by ``prioRules`` is discarded at MVP.py:46), then the
  per-aircraft finalize (67-143).
* ``mvp_pair``  MVP.py:149-231 -- one pair's dv and tsolV.
* ``prio_rules`` MVP.py:235-300 -- FF1/FF2/FF3/LAY1/LAY2, first output only.

Pairs are addressed by index (``ci``/``cj``) instead of ``traf.id.index``
(ids are unique in BlueSky's Traffic, so both address the same aircraft).
"""
import numpy as np

FT = 0.3048        # bluesky/tools/aero.py:12
NM = 1852.0        # bluesky/tools/aero.py:16


def params_from_settings(R, dh, dtlookahead, mar, swresohoriz=True, swresospd=False,
                         swresohdg=False, swresovert=False, swprio=False, priocode='FF1',
                         vmin_kts=200.0, vmax_kts=500.0):
    """ASAS scalars as set in asas.py:81-103."""
    return dict(Rm=R * mar, dhm=dh * mar, dtlookahead=dtlookahead,
                vmin=vmin_kts * NM / 3600., vmax=vmax_kts * NM / 3600.,
                vsmin=-3000. / 60. * FT, vsmax=3000. / 60. * FT,
                swresohoriz=bool(swresohoriz), swresospd=bool(swresospd),
                swresohdg=bool(swresohdg), swresovert=bool(swresovert),
                swprio=bool(swprio), priocode=priocode)


def mvp_pair(p, qdr, dist, tcpa, tLOS, alt1, alt2, v1, v2):
    """MVP.py:149-231 for one pair; v1/v2 = (gseast, gsnorth, vs)."""
    qdr = np.radians(qdr)
    drel = np.array([np.sin(qdr) * dist, np.cos(qdr) * dist, alt2 - alt1])
    vrel = np.array(np.asarray(v2) - np.asarray(v1))

    dcpa = drel + vrel * tcpa
    dabsH = np.sqrt(dcpa[0] * dcpa[0] + dcpa[1] * dcpa[1])
    iH = p['Rm'] - dabsH
    if dabsH <= 10.:
        dabsH = 10.
        dcpa[0] = drel[1] / dist * dabsH
        dcpa[1] = -drel[0] / dist * dabsH

    dv1 = (iH * dcpa[0]) / (abs(tcpa) * dabsH)
    dv2 = (iH * dcpa[1]) / (abs(tcpa) * dabsH)
    if p['Rm'] < dist and dabsH < dist:
        erratum = np.cos(np.arcsin(p['Rm'] / dist) - np.arcsin(dabsH / dist))
        dv1 = dv1 / erratum
        dv2 = dv2 / erratum

    iV = p['dhm'] if abs(vrel[2]) > 0.0 else p['dhm'] - abs(drel[2])
    tsolV = abs(drel[2] / vrel[2]) if abs(vrel[2]) > 0.0 else tLOS
    if tsolV > p['dtlookahead']:
        tsolV = tLOS
        iV = p['dhm']
    with np.errstate(divide='ignore', invalid='ignore'):
        dv3 = np.where(abs(vrel[2]) > 0.0, (iV / tsolV) * (-vrel[2] / abs(vrel[2])), (iV / tsolV))
    return np.array([dv1, dv2, dv3]), tsolV


def prio_rules(code, vs1, vs2, dv_mvp, dv1):
    """MVP.py:235-300; returns the new dv1 (dv2 is discarded by the caller)."""
    if code == "FF1":
        dv_mvp[2] = dv_mvp[2] / 2.0
        dv1 = dv1 - dv_mvp
    if code == "FF2":
        dv_mvp[2] = dv_mvp[2] / 2.0
        if abs(vs1) < 0.1 and abs(vs2) > 0.1:
            pass
        elif abs(vs2) < 0.1 and abs(vs1) > 0.1:
            dv1 = dv1 - dv_mvp
        else:
            dv1 = dv1 - dv_mvp
    elif code == "FF3":
        if abs(vs1) < 0.1 and abs(vs2) > 0.1:
            dv_mvp[2] = 0.0
            dv1 = dv1 - dv_mvp
        elif abs(vs2) < 0.1 and abs(vs1) > 0.1:
            dv_mvp[2] = 0.0
        else:
            dv_mvp[2] = dv_mvp[2] / 2.0
            dv1 = dv1 - dv_mvp
    elif code == "LAY1":
        dv_mvp[2] = 0.0
        if abs(vs1) < 0.1 and abs(vs2) > 0.1:
            pass
        elif abs(vs2) < 0.1 and abs(vs1) > 0.1:
            dv1 = dv1 - dv_mvp
        else:
            dv1 = dv1 - dv_mvp
    elif code == "LAY2":
        dv_mvp[2] = 0.0
        if abs(vs1) < 0.1 and abs(vs2) > 0.1:
            dv1 = dv1 - dv_mvp
        elif abs(vs2) < 0.1 and abs(vs1) > 0.1:
            pass
        else:
            dv1 = dv1 - dv_mvp
    return dv1


def resolve_arrays(ci, cj, qdr, dist, tcpa, tLOS, gseast, gsnorth, vs, alt, trk, gs,
                   selalt, apvs, asasalt, params, noreso=None, resooff=None):
    """MVP.resolve (MVP.py:14-143) on index arrays.

    ``noreso``/``resooff``: optional per-aircraft bool masks standing for
    ``asas.noresolst``/``asas.resoofflst`` membership with the switch on.
    ``asasalt`` is the persistent ``asas.alt`` (read-modify-write).
    Returns dict(trk, tas, vs, alt, asase, asasn, timesolveV).
    """
    p = params
    n = len(alt)
    dv = np.zeros((n, 3))
    asasn = np.zeros(n, dtype=np.float32)
    asase = np.zeros(n, dtype=np.float32)
    timesolveV = np.ones(n) * 1e9

    for k in range(len(ci)):
        id1 = int(ci[k])
        id2 = int(cj[k])
        v1 = np.array([gseast[id1], gsnorth[id1], vs[id1]])
        v2 = np.array([gseast[id2], gsnorth[id2], vs[id2]])
        dv_mvp, tsolV = mvp_pair(p, qdr[k], dist[k], tcpa[k], tLOS[k], alt[id1], alt[id2], v1, v2)
        if tsolV < timesolveV[id1]:
            timesolveV[id1] = tsolV
        if p['swprio']:
            dv[id1] = prio_rules(p['priocode'], vs[id1], vs[id2], dv_mvp, dv[id1])
        else:
            dv_mvp[2] = 0.5 * dv_mvp[2]
            dv[id1] = dv[id1] - dv_mvp
        if noreso is not None and noreso[id2]:
            dv[id1] = dv[id1] + dv_mvp
        if resooff is not None and resooff[id1]:
            dv[id1] = 0.0

    dv = np.transpose(dv)
    v = np.array([gseast, gsnorth, vs])
    newv = dv + v
    ids = dv[0, :] ** 2 + dv[1, :] ** 2 > 0

    if p['swresohoriz']:
        if p['swresospd'] and not p['swresohdg']:
            newtrack = trk
            newgs = np.sqrt(newv[0, :] ** 2 + newv[1, :] ** 2)
            newvs = vs
        elif p['swresohdg'] and not p['swresospd']:
            newtrack = (np.arctan2(newv[0, :], newv[1, :]) * 180 / np.pi) % 360
            newgs = gs
            newvs = vs
        else:
            newtrack = (np.arctan2(newv[0, :], newv[1, :]) * 180 / np.pi) % 360
            newgs = np.sqrt(newv[0, :] ** 2 + newv[1, :] ** 2)
            newvs = vs
    elif p['swresovert']:
        newtrack = trk
        newgs = gs
        newvs = newv[2, :]
    else:
        newtrack = (np.arctan2(newv[0, :], newv[1, :]) * 180 / np.pi) % 360
        newgs = np.sqrt(newv[0, :] ** 2 + newv[1, :] ** 2)
        newvs = newv[2, :]

    newgscapped = np.maximum(p['vmin'], np.minimum(p['vmax'], newgs))
    vscapped = np.maximum(p['vsmin'], np.minimum(p['vsmax'], newvs))

    a_trk = newtrack
    a_tas = newgscapped
    a_vs = vscapped
    asase[ids] = a_tas[ids] * np.sin(a_trk[ids] / 180 * np.pi)
    asasn[ids] = a_tas[ids] * np.cos(a_trk[ids] / 180 * np.pi)

    a_alt = asasalt
    signdvs = np.sign(a_vs - apvs * np.sign(selalt - alt))
    signalt = np.sign(a_alt - selalt)
    a_alt = np.where(np.logical_or(signdvs == 0, signdvs == signalt), a_alt, selalt)

    altCondition = np.logical_and(timesolveV < p['dtlookahead'], np.abs(dv[2, :]) > 0.0)
    asasalttemp = a_vs * timesolveV + alt
    a_alt[altCondition] = asasalttemp[altCondition]
    a_alt = a_alt * (1 - p['swresohoriz']) + selalt * p['swresohoriz']

    return dict(trk=np.asarray(a_trk, dtype=np.float64), tas=a_tas, vs=a_vs, alt=a_alt,
                asase=asase, asasn=asasn, timesolveV=timesolveV)
