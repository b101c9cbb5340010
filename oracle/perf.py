"""OpenAP flight phase, phase-dependent envelope and acceleration
(bluesky/traffic/performance/openap/phase.py:14-66, perfoap.py:115-131,
211-262, 271-280).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

``OpenAP.update`` (perfoap.py:115-131) runs every step between
Pilot.APorASAS and Pilot.applylimits (traffic.py:397-404): the phase is
inferred from the pre-step tas / vs / alt, the six envelope columns are
looked up per aircraft type and phase, and ``acceleration()`` (read by
UpdateAirSpeed, traffic.py:429) is 2 m/s^2 on the ground, 0.5 otherwise.
The envelope is restated here from the reference's coefficient dicts
(``Coefficient.limits_fixwing`` / ``limits_rotor``, coeff.py:80-131), not
from the product's type table, so the table builder is checked too.
"""
import numpy as np

NA, TO, IC, CL, CR, DE, AP, LD, GD = range(9)   # phase.py:4-12
LIFT_FIXWING, LIFT_ROTOR = 1, 2                  # coeff.py:9-10


def phase_fixwing(roc_si, alt_si):
    """phase.get_fixwing (phase.py:31-62), unit 'SI' (speed is not used)."""
    roc = roc_si / 0.00508
    alt = alt_si / 0.3048
    ph = np.zeros(len(roc), dtype=int)
    ph[(alt <= 10) & (roc <= 100) & (roc >= -100)] = GD
    ph[(alt >= 0) & (alt <= 1000) & (roc >= 0)] = IC
    ph[(alt >= 0) & (alt <= 1000) & (roc <= 0)] = AP
    ph[(alt >= 1000) & (roc >= 100)] = CL
    ph[(alt >= 1000) & (roc <= -100)] = DE
    ph[(alt >= 5000) & (roc <= 100) & (roc >= -100)] = CR
    return ph


def phase(lifttype, tas, vs, alt):
    """phase.get (phase.py:14-29): fixwing rule, rotors NA (a float array as
    the reference's np.where returns)."""
    ph = np.zeros(len(tas))
    ph = np.where(lifttype == LIFT_FIXWING, phase_fixwing(vs, alt), ph)
    ph = np.where(lifttype == LIFT_ROTOR, np.ones(len(tas)) * NA, ph)
    return ph


def limit_matrix(limits_fixwing, limits_rotor, actypes, lifttype, phases):
    """OpenAP.__construct_limit_matrix (perfoap.py:211-262): n x 6
    [vmin, vmax, vsmin, vsmax, hmax, axmax] (rotors leave axmax 0)."""
    lim = np.zeros((len(actypes), 6))
    wing = np.unique(actypes[np.where(lifttype == LIFT_FIXWING)[0]])
    for mdl in wing:
        c = limits_fixwing[mdl]
        m = actypes == mdl
        for ph, v in ((NA, 0), (TO, c['vminto']), (IC, c['vminic']), ((CL, CR, DE), c['vminer']),
                      (AP, c['vminap']), (LD, c['vminld']), (GD, 0)):
            sel = np.isin(phases, ph)
            lim[:, 0] = np.where(m & sel, v, lim[:, 0])
        for ph, v in ((NA, c['vmaxer']), (TO, c['vmaxto']), (IC, c['vmaxic']), ((CL, CR, DE), c['vmaxer']),
                      (AP, c['vmaxap']), (LD, c['vmaxld']), (GD, c['vmaxer'])):
            sel = np.isin(phases, ph)
            lim[:, 1] = np.where(m & sel, v, lim[:, 1])
        lim[:, 2] = np.where(m, c['vsmin'], lim[:, 2])
        lim[:, 3] = np.where(m, c['vsmax'], lim[:, 3])
        lim[:, 4] = np.where(m, c['hmax'], lim[:, 4])
        lim[:, 5] = np.where(m, c['axmax'], lim[:, 5])
    rot = np.unique(actypes[np.where(lifttype == LIFT_ROTOR)[0]])
    for mdl in rot:
        c = limits_rotor[mdl]
        m = actypes == mdl
        for col, key in enumerate(('vmin', 'vmax', 'vsmin', 'vsmax', 'hmax')):
            lim[:, col] = np.where(m, c[key], lim[:, col])
    return lim


def envelope(lim):
    """limit matrix -> the dict oracle.kinematics.openap_limits reads."""
    return dict(vmin=lim[:, 0], vmax=lim[:, 1], vsmin=lim[:, 2], vsmax=lim[:, 3], hmax=lim[:, 4],
                axmax=lim[:, 5])


def acceleration(phases):
    """OpenAP.acceleration (perfoap.py:271-280)."""
    accs = np.zeros(len(phases))
    accs[phases == GD] = 2
    accs[phases != GD] = 0.5
    return accs
