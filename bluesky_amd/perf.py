"""OpenAP flight-phase envelope for the resident step.

``OpenAP.update`` (bluesky/traffic/performance/openap/perfoap.py:115-131)
re-derives every aircraft's flight phase from tas / vs / alt each step
(phase.py:14-62) and looks its speed / vertical-speed / altitude /
acceleration envelope up per aircraft type and phase
(``__construct_limit_matrix``, perfoap.py:211-262); ``acceleration()``
(perfoap.py:271-280) is 2 m/s^2 on the ground, 0.5 otherwise.  On the device
(``bsa_sim_set_perf``) this runs inside K4' of every step: the host hands
over one row per aircraft type and a type index per aircraft, built here from
the reference's own coefficient object (``bs.traf.perf.coeff``,
coeff.py:23-131) and per-aircraft ``perf.actypes`` / ``perf.lifttype``.

Table row (``PERF_COLS`` doubles): vmin by phase NA..GD (9), vmax by phase
(9), vsmin, vsmax, hmax, axmax, lifttype, 0.
"""
import numpy as np

NA, TO, IC, CL, CR, DE, AP, LD, GD = range(9)   # phase.py:4-12
LIFT_FIXWING, LIFT_ROTOR = 1, 2                  # coeff.py:9-10
PERF_COLS = 24


def _fixwing_row(c):
    """perfoap.py:232-250: the speed limits of a fixed-wing type per phase."""
    vmin = [0.0, c['vminto'], c['vminic'], c['vminer'], c['vminer'], c['vminer'], c['vminap'], c['vminld'], 0.0]
    vmax = [c['vmaxer'], c['vmaxto'], c['vmaxic'], c['vmaxer'], c['vmaxer'], c['vmaxer'], c['vmaxap'],
            c['vmaxld'], c['vmaxer']]
    return vmin + vmax + [c['vsmin'], c['vsmax'], c['hmax'], c['axmax'], float(LIFT_FIXWING), 0.0]


def _rotor_row(c):
    """perfoap.py:254-261: rotor limits do not depend on the phase; axmax is
    never set for rotors (0)."""
    return [c['vmin']] * 9 + [c['vmax']] * 9 + [c['vsmin'], c['vsmax'], c['hmax'], 0.0, float(LIFT_ROTOR), 0.0]


def type_table(limits_fixwing, limits_rotor, actypes, lifttype):
    """(table float64 [ntypes, PERF_COLS], type index int32 [n]) for the
    aircraft types ``actypes`` (str per aircraft, as ``perf.actypes``) with
    lift types ``lifttype`` (``perf.lifttype``).  ``limits_*``: the
    reference's ``Coefficient.limits_fixwing`` / ``limits_rotor`` dicts.
    Aircraft with another lift type get a row of zeros with lifttype 0 (the
    reference's limit matrix leaves them 0, phase.get gives them NA)."""
    actypes = np.asarray(actypes).astype(str)
    lifttype = np.asarray(lifttype).astype(np.int64)
    keys = sorted(set(zip(actypes.tolist(), lifttype.tolist())))
    rows = []
    for mdl, lt in keys:
        if lt == LIFT_FIXWING:
            rows.append(_fixwing_row(limits_fixwing[mdl]))
        elif lt == LIFT_ROTOR:
            rows.append(_rotor_row(limits_rotor[mdl]))
        else:
            rows.append([0.0] * PERF_COLS)
    where = {k: i for i, k in enumerate(keys)}
    tidx = np.array([where[k] for k in zip(actypes.tolist(), lifttype.tolist())], dtype=np.int32)
    return np.array(rows, dtype=np.float64).reshape(len(keys), PERF_COLS), tidx


def from_openap(perf):
    """Table + type index straight from a reference ``OpenAP`` instance
    (``bs.traf.perf``)."""
    return type_table(perf.coeff.limits_fixwing, perf.coeff.limits_rotor, perf.actypes, perf.lifttype)
