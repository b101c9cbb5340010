"""ASAS.update bookkeeping and ResumeNav (bluesky/traffic/asas/asas.py:409-504).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Pairs are index tuples (idx1, idx2) instead of callsign tuples (ids are
unique, so the sets correspond one to one).  One call = the part of
``ASAS.update`` after detect / resolve:

* ``resopairs.update(confpairs)``                         asas.py:490
* ``confpairs_unique = {frozenset(p) ...}`` (and LoS)     asas.py:494-495
* ``confpairs_all.extend(unique - previous unique)``      asas.py:497-498
* ``ResumeNav()``                                         asas.py:409-471,504

Deleted aircraft (Traffic.delete, traffic.py:364-378): the reference's sets
are keyed by callsign and untouched by a delete; ``delete()`` / ``create()``
restate that on indices -- a pair of a deleted ownship goes (ResumeNav drops it
at the next call, asas.py:420-422, before anything reads it), a pair whose
intruder was deleted becomes (i, -1) and is dropped by the next ResumeNav with
``active[i] = False`` (idx2 < 0, asas.py:454-468), and previous-call unique
pairs with a deleted member can never match again, so they go.

ResumeNav per resopair:
flat-earth ``dist`` vector (re = 6371000, cos of the mean latitude),
``past_cpa = dot(dist, vrel) > 0``, ``hor_los = |dist| < R``,
``is_bouncing = |trk1 - trk2| < 30 and |dist| < Rm``; keep the pair and set
``active[idx1] = True`` iff ``not past_cpa or hor_los or is_bouncing``, else
set ``active[idx1] = False`` and drop the pair.  The reference iterates a
Python set, so an aircraft with pairs of BOTH outcomes ends with the value of
whichever pair the hash order visits last; this restatement (and the GPU)
uses the order-free rule "active iff any of its pairs is kept", which equals
the reference whenever an aircraft's pairs agree (``ambiguous()`` lists the
others).  Waypoint recovery (``route.direct``, asas.py:459-462) is autopilot
state and out of scope.
"""
import numpy as np

RE = 6371000.     # asas.py:426


def pair_keep(i, j, lat, lon, gseast, gsnorth, trk, R, Rm):
    """ResumeNav's decision for resopair (i, j) (asas.py:424-452); j < 0: the
    intruder was deleted -- recovery starts (asas.py:454-468)."""
    if j < 0:
        return False
    dist = RE * np.array([np.radians(lon[j] - lon[i]) * np.cos(0.5 * np.radians(lat[j] + lat[i])),
                          np.radians(lat[j] - lat[i])])
    vrel = np.array([gseast[j] - gseast[i], gsnorth[j] - gsnorth[i]])
    past_cpa = np.dot(dist, vrel) > 0.0
    hdist = np.linalg.norm(dist)
    hor_los = hdist < R
    is_bouncing = abs(trk[i] - trk[j]) < 30.0 and hdist < Rm
    return bool(not past_cpa or hor_los or is_bouncing)


class Bookkeeping:
    """The ASAS sets of one simulation, updated once per CD call."""

    def __init__(self, n):
        self.resopairs = set()
        self.confpairs_unique = set()
        self.lospairs_unique = set()
        self.confpairs_all = 0   # lengths of the reference's cumulative lists
        self.lospairs_all = 0
        self.active = np.zeros(n, dtype=bool)
        self.last_keep = {}

    def update(self, confpairs, lospairs, lat, lon, gseast, gsnorth, trk, R, Rm):
        """confpairs / lospairs: iterables of (i, j); state arrays of this step."""
        confpairs = [tuple(map(int, p)) for p in confpairs]
        lospairs = [tuple(map(int, p)) for p in lospairs]
        self.resopairs.update(confpairs)
        cu = {frozenset(p) for p in confpairs}
        lu = {frozenset(p) for p in lospairs}
        self.confpairs_all += len(cu - self.confpairs_unique)
        self.lospairs_all += len(lu - self.lospairs_unique)
        self.confpairs_unique, self.lospairs_unique = cu, lu
        # ResumeNav
        keep = {p: pair_keep(p[0], p[1], lat, lon, gseast, gsnorth, trk, R, Rm)
                for p in self.resopairs}
        rows = {}
        for (i, j), k in keep.items():
            rows[i] = rows.get(i, False) or k
        for i, a in rows.items():
            self.active[i] = a
        self.resopairs = {p for p, k in keep.items() if k}
        self.last_keep = keep
        return keep

    def delete(self, idx):
        """np.delete of aircraft ``idx`` (the rest shift down in order)."""
        n = len(self.active)
        gone = np.zeros(n, dtype=bool)
        gone[np.asarray(idx, dtype=np.int64)] = True
        new = np.cumsum(~gone) - 1
        new[gone] = -1
        self.resopairs = {(int(new[i]), -1 if j < 0 else int(new[j])) for i, j in self.resopairs if not gone[i]}
        remap = lambda s: {frozenset(int(new[x]) for x in p) for p in s if not any(gone[x] for x in p)}
        self.confpairs_unique = remap(self.confpairs_unique)
        self.lospairs_unique = remap(self.lospairs_unique)
        self.active = self.active[~gone]

    def create(self, m):
        """Traffic.create of m aircraft (appended, asas.active False)."""
        self.active = np.concatenate([self.active, np.zeros(m, dtype=bool)])

    def ambiguous(self, keep):
        """Aircraft whose resopairs disagree (reference result hash-order dependent)."""
        seen = {}
        for (i, _), k in keep.items():
            seen.setdefault(i, set()).add(k)
        return sorted(i for i, s in seen.items() if len(s) > 1)
