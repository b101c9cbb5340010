"""Synthetic traffic generator used by bench.py and the tests.

``rng = np.random.default_rng(seed)``; draw order lat, lon, alt, trk, gs, vs.

* box(L NM) centred on 52N 4E: ``lat = 52 + (U-0.5) L/60``,
  ``lon = 4 + (U-0.5) (L/60)/cos(52 deg)``
* global: ``lat = degrees(arcsin(U(-0.94, 0.94)))`` (|lat| <= 70 deg, uniform
  on the sphere), ``lon = U(-180, 180)``
* ``alt = U(100, 400) * 100 ft`` (FL100-400, metres), ``trk = U(0, 360)``,
  ``gs = U(200, 500) kts``, ``vs = 0`` with p = 0.7 else ``+-U(2.5, 12.5)`` m/s
  (draws: ``random() < 0.7``, ``uniform(2.5, 12.5)``, ``choice([-1, 1])`` --
  reproduces SURVEY.md 9's probe count, 14 317 confpairs at box10k seed 7)
* ``id = 'A%06d'``

Units follow BlueSky's Traffic arrays (deg, m, m/s).  The density-matched
100k box is 1581 NM (same aircraft per area as 10k in 500 NM).
"""
import numpy as np

FT = 0.3048           # bluesky/tools/aero.py:12
KTS = 0.514444        # bluesky/tools/aero.py:11
NM = 1852.0           # bluesky/tools/aero.py:16

# default CD settings (bluesky/traffic/asas/asas.py:10-13, data/default.cfg)
RPZ = 5.0 * NM        # asas_pzr = 5 nm
HPZ = 1000.0 * FT     # asas_pzh = 1000 ft
TLOOKAHEAD = 300.0    # asas_dtlookahead [s]


class Traffic:
    """Minimal duck-typed stand-in for ``bs.traf`` (the attributes detect reads)."""

    def __init__(self, lat, lon, alt, trk, gs, vs, ids=None):
        self.lat = np.ascontiguousarray(lat, dtype=np.float64)
        self.lon = np.ascontiguousarray(lon, dtype=np.float64)
        self.alt = np.ascontiguousarray(alt, dtype=np.float64)
        self.trk = np.ascontiguousarray(trk, dtype=np.float64)
        self.gs = np.ascontiguousarray(gs, dtype=np.float64)
        self.vs = np.ascontiguousarray(vs, dtype=np.float64)
        self.ntraf = len(self.lat)
        self.id = ids if ids is not None else ['A%06d' % i for i in range(self.ntraf)]

    def as_dict(self):
        return dict(lat=self.lat, lon=self.lon, alt=self.alt, trk=self.trk,
                    gs=self.gs, vs=self.vs, id=self.id)


def _kinematics(rng, n):
    alt = rng.uniform(100.0, 400.0, n) * 100.0 * FT
    trk = rng.uniform(0.0, 360.0, n)
    gs = rng.uniform(200.0, 500.0, n) * KTS
    level = rng.random(n) < 0.7
    mag = rng.uniform(2.5, 12.5, n)
    sgn = rng.choice([-1.0, 1.0], n)   # the survey probe's draw: 14 317 / 2 228 pairs at box10k
    vs = np.where(level, 0.0, mag * sgn)
    return alt, trk, gs, vs


def box(n, L_nm=500.0, seed=7, lat0=52.0, lon0=4.0):
    """n aircraft uniformly in an L x L NM box around (lat0, lon0)."""
    rng = np.random.default_rng(seed)
    lat = lat0 + (rng.random(n) - 0.5) * L_nm / 60.0
    lon = lon0 + (rng.random(n) - 0.5) * (L_nm / 60.0) / np.cos(np.radians(lat0))
    alt, trk, gs, vs = _kinematics(rng, n)
    return Traffic(lat, lon, alt, trk, gs, vs)


def density_matched_box_nm(n, n_ref=10000, L_ref=500.0):
    """Box side giving the same density as n_ref aircraft in L_ref NM."""
    return L_ref * np.sqrt(n / n_ref)


def global_traffic(n, seed=7):
    """n aircraft uniform on the sphere with |lat| <= ~70 deg."""
    rng = np.random.default_rng(seed)
    lat = np.degrees(np.arcsin(rng.uniform(-0.94, 0.94, n)))
    lon = rng.uniform(-180.0, 180.0, n)
    alt, trk, gs, vs = _kinematics(rng, n)
    return Traffic(lat, lon, alt, trk, gs, vs)


def workload(name, n=None, seed=7):
    """Named workloads from BASELINE.json ``configs``."""
    if name == 'box10k':
        return box(n or 10000, 500.0, seed)
    if name == 'box100k':
        n = n or 100000
        return box(n, density_matched_box_nm(n), seed)
    if name == 'global1m':
        return global_traffic(n or 1000000, seed)
    raise ValueError('unknown workload %r' % name)
