"""Shared helpers for the parity tests (fixtures live in tests/golden/)."""
import glob
import os

import numpy as np

from bluesky_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

# Parity tolerance for fp64 outputs (north_star: "within 1e-9 relative").
# |got - exp| <= RTOL * max(|got|, |exp|) + RTOL * SCALE[field]; the absolute
# floor (1e-9 of the quantity's natural scale) only matters where the value
# itself is ~0 through cancellation (e.g. tcpa of a pair at its CPA).
RTOL = 1e-9


def golden(pattern):
    return sorted(glob.glob(os.path.join(GOLDEN, pattern)))


def case_name(path):
    return os.path.basename(path)[:-4]


def load_cd(path):
    z = dict(np.load(path, allow_pickle=False))
    own = synth.Traffic(z['lat'], z['lon'], z['alt'], z['trk'], z['gs'], z['vs'])
    intr = own
    if not bool(z['same']):
        intr = synth.Traffic(z['ilat'], z['ilon'], z['ialt'], z['itrk'], z['igs'], z['ivs'])
    return own, intr, z


def close(got, exp, scale, rtol=RTOL):
    got = np.asarray(got, dtype=np.float64)
    exp = np.asarray(exp, dtype=np.float64)
    if got.shape != exp.shape:
        return False, 'shape %s != %s' % (got.shape, exp.shape)
    both_nan = np.isnan(got) & np.isnan(exp)
    same_inf = np.isinf(got) & np.isinf(exp) & (np.sign(got) == np.sign(exp))
    err = np.abs(got - exp)
    tol = rtol * np.maximum(np.abs(got), np.abs(exp)) + rtol * scale
    bad = ~(both_nan | same_inf | (err <= tol))
    if bad.any():
        k = np.flatnonzero(bad)[0]
        return False, '%d mismatches, first at %d: got %r exp %r' % (bad.sum(), k, got[k], exp[k])
    return True, ''


def assert_detect_equal(got, exp, rpz, tla, rows=None):
    """Pair sets/orders exact, inconf exact, reals within RTOL."""
    for k in ('ci', 'cj', 'li', 'lj'):
        g = np.asarray(got[k], dtype=np.int64)
        e = np.asarray(exp[k], dtype=np.int64)
        assert g.shape == e.shape and np.array_equal(g, e), \
            '%s differs: got %d entries, expected %d' % (k, len(g), len(e))
    assert np.array_equal(np.asarray(got['inconf']).astype(bool), np.asarray(exp['inconf']).astype(bool))
    scales = dict(qdr=360.0, dist=rpz, tcpa=tla, tinconf=tla, tcpamax=tla)
    for k, s in scales.items():
        ok, msg = close(got[k], exp[k], s)
        assert ok, '%s: %s' % (k, msg)


TRACE_PAIRS = {'ci': 'ci', 'cj': 'ci', 'qdr': 'ci', 'dist': 'ci', 'tcpa': 'ci', 'tLOS': 'ci',
               'li': 'li', 'lj': 'li', 'reso_i': 'reso_i', 'reso_j': 'reso_i',
               'reso_in_i': 'reso_in_i', 'reso_in_j': 'reso_in_i'}


def load_trace(path):
    """Full-simulator trace (tools/make_trace.py): (settings dict, list of per-ASAS-call
    dicts).  Per call: the traffic state the detector read (lat lon trk gs alt vs tas
    gseast gsnorth selalt apvs), asas.alt / asas.active before the call, the detect
    outputs (ci cj li lj inconf tcpamax qdr dist tcpa tLOS), asas.trk/tas/vs/alt and
    asase/asasn after it, resopairs before / after, asas.active after, the four
    bookkeeping counts and whether MVP ran; with created / deleted traffic also
    the callsigns (``ids``) and per-aircraft arrays of varying length."""
    z = dict(np.load(path, allow_pickle=False))
    n = int(z['ncalls'])
    settings = {k[4:]: z[k][()] for k in z if k.startswith('set_')}
    calls = []
    for c in range(n):
        rec = {}
        for k, v in z.items():
            if k.startswith('set_') or k == 'ncalls' or k.endswith('_off'):
                continue
            if k + '_off' in z or k in TRACE_PAIRS:  # concatenated over calls
                off = z[k + '_off'] if k + '_off' in z else z[TRACE_PAIRS[k] + '_off']
                rec[k] = v[off[c]:off[c + 1]]
            else:                                     # stacked [call, ...]
                rec[k] = v[c]
        calls.append(rec)
    return settings, calls
