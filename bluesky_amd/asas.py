"""Drop-in ``ASAS.update`` on MI355X: one ASAS call -- detection, resolution
and the conflict bookkeeping -- on the device (``asas.py:473-504``, with
``ResumeNav``, ``asas.py:409-471``).

The reference's ``ASAS.update`` runs the detector and resolver plugins and
then keeps its bookkeeping in Python sets of callsign tuples: ``resopairs``,
``confpairs_unique`` / ``lospairs_unique`` (frozensets of every pair, rebuilt
each call) and the cumulative ``confpairs_all`` / ``lospairs_all``, followed by
``ResumeNav``'s loop over every resopair with ``id2idx`` lookups
(``asas.py:417-471,490-502``) -- ~1.5e5 tuples per call at 100k aircraft.
Here the whole call is one ``bsa_sim_cd`` on the GPU-resident sim
(``bsa_sim.hip`` / ``bsa_asas.hip``): the host simulator's traffic is written
with ``bsa_sim_update`` (its autopilot, performance model and stack ran in
between, ``traffic.py:383-404``), then detect -> MVP (or the default CR OFF =
``DoNothing.resolve``) -> resopairs merge -> ``ResumeNav``'s past-CPA /
horizontal-LoS / bouncing test -> unique / cumulative counts, all on the
device.  The ASAS object then carries the reference's attributes:

* ``confpairs`` / ``lospairs``: row-major lists of ``(id_i, id_j)`` tuples
  (``StateBasedCD.py:93-101``), built only when read (``len()`` and truth value
  are free); ``inconf``, ``tcpamax``, ``qdr``, ``dist``, ``tcpa``, ``tLOS``;
* ``trk`` / ``tas`` / ``vs`` / ``alt`` / ``asase`` / ``asasn`` as the resolver
  left them, ``active`` as ``ResumeNav`` left it (the reference's value for an
  aircraft whose resopairs disagree depends on Python set order; the device
  gives "active iff any pair is kept");
* ``resopairs``, ``confpairs_unique``, ``lospairs_unique``: sets whose ``len()``
  comes from the device and whose members are built on first use;
  ``confpairs_all`` / ``lospairs_all``: ``len()`` from the device; their members
  only with ``history=True`` (which builds the reference's Python sets every
  call and costs what the reference costs);
* ``ResumeNav``'s waypoint recovery (``route.direct`` for an ownship whose pair
  was dropped, ``asas.py:459-462``) is applied on the host from the device's
  per-aircraft drop flags.

Install once after ``bs.init()`` (before the first ASAS call)::

    import bluesky as bs
    from bluesky_amd import asas as gasas
    gasas.install(bs.traf.asas, bs.traf)

Supported: the StateBased detector (``CDMETHOD STATEBASED`` or ``GPU``) with
CR ``OFF`` (``DoNothing``) or ``MVP`` / ``GPUMVP``; every MVP switch, NORESO /
RESOOFF lists, stack changes of ZONER / ZONEDH / DTLOOK between calls, and
Traffic create / delete between calls (mirrored with ``bsa_sim_create`` /
``bsa_sim_delete``, which keep the bookkeeping of the other aircraft).  Any
other CD / CR method raises ``NotImplementedError`` -- there is no CPU path.
One rank only: BlueSky's ``ASAS.update`` is one process's call over the whole
traffic, so a context joined to a communicator or group (several ranks, each
holding only its rows' outputs) raises ``NotImplementedError``.
"""
import collections.abc
import time
import warnings

import numpy as np

from . import _lib, mvp, statebased

_ZEROS = ('bank', 'eps', 'accel')


class PairList(collections.abc.Sequence):
    """``asas.confpairs`` / ``lospairs``: the reference's list of ``(id_i, id_j)``
    tuples in row-major order, materialised from the index arrays on first
    element access (``len()`` / truth value need no tuples)."""

    __slots__ = ('_ids', 'i', 'j', '_list')

    def __init__(self, ids, i, j):
        self._ids, self.i, self.j, self._list = ids, i, j, None

    def _mat(self):
        if self._list is None:
            self._list = statebased.pairs_from_indices(self._ids, self.i, self.j)
        return self._list

    def __len__(self):
        return len(self.i)

    def __getitem__(self, k):
        return self._mat()[k]

    def __iter__(self):
        return iter(self._mat())

    def __eq__(self, other):
        if isinstance(other, (list, tuple, PairList)):
            return list(self) == list(other)
        return NotImplemented

    __hash__ = None

    def __repr__(self):
        return 'PairList(%r)' % (self._mat(),)


class _LazySet(collections.abc.Set):
    """A set whose size the device counted; its members are built on first use."""

    def __init__(self, count, build):
        self._count, self._build, self._set = int(count), build, None

    @classmethod
    def _from_iterable(cls, it):
        return set(it)   # set algebra (a - b, a | b, ...) yields plain sets, as on the reference's

    def _mat(self):
        if self._set is None:
            self._set = self._build()
        return self._set

    def __len__(self):
        return self._count

    def __iter__(self):
        return iter(self._mat())

    def __contains__(self, x):
        return x in self._mat()

    def __repr__(self):
        return '%s(%r)' % (type(self).__name__, self._mat())


class UniquePairs(_LazySet):
    """``confpairs_unique`` / ``lospairs_unique``: ``{frozenset(p) for p in pairs}``
    (``asas.py:494-495``) with the device's count."""

    def __init__(self, count, pairs):
        super().__init__(count, lambda: {frozenset(p) for p in pairs})


class ResoPairs(_LazySet):
    """``resopairs``: the device's resopairs as ``(id1, id2)`` callsign tuples; a pair
    whose intruder was deleted since the last call reads ``(id1, None)``."""


class PairHistory(collections.abc.Sequence):
    """``confpairs_all`` / ``lospairs_all`` without recorded history: ``len()`` is the
    device's cumulative count (what ScreenIO reads, ``screenio.py:207-210``);
    the members were not kept (``install(..., history=True)`` keeps them)."""

    def __init__(self, count):
        self._count = int(count)

    def __len__(self):
        return self._count

    def __getitem__(self, k):
        raise RuntimeError('pair history not recorded: install the ASAS drop-in with history=True')

    def __repr__(self):
        return 'PairHistory(len=%d)' % self._count


def _module_name(m):
    return getattr(m, '__name__', type(m).__name__)


class DeviceASAS:
    """The device-side replacement of one ``ASAS`` instance's ``update``."""

    def __init__(self, asas, traf, ctx=None, history=False, waypoint_recovery=True):
        self.asas, self.traf = asas, traf
        self.ctx = ctx or _lib.default_context()
        if getattr(self.ctx, 'comm_rank_world', (0, 1))[1] > 1:
            raise NotImplementedError('ASAS drop-in: one rank only (this context is rank %d of %d; '
                                      'the per-rank outputs cover only its rows)' % self.ctx.comm_rank_world)
        self.history = history
        self.waypoint_recovery = waypoint_recovery
        self._ids = None        # callsigns of the device's traffic, in index order
        self._idarr = None      # the same as an object array (tuple building)
        self._reso = None       # the resopairs object last set on asas (reset detection)
        self._base = [0, 0]     # confpairs_all / lospairs_all counted before the last re-init
        self._prev_unique = (set(), set())   # history=True: last call's unique sets
        self.timings = {}       # wall time [s] of the last call's phases (bench.py's asas_update line)

    # ------------------------------------------------------------- plumbing
    def _reso_mode(self):
        """1: MVP on the device, 0: the default CR OFF (DoNothing.resolve)."""
        cr = self.asas.cr
        name = _module_name(cr)
        if cr is mvp or name.endswith('MVP'):
            return 1
        if name.endswith('DoNothing'):
            return 0
        raise NotImplementedError('ASAS drop-in: CR method %s has no device implementation '
                                  '(supported: OFF, MVP, GPUMVP)' % name)

    def _check_cd(self):
        cd = self.asas.cd
        name = _module_name(cd)
        if not (cd is statebased or name.endswith('StateBasedCD') or
                isinstance(cd, statebased.ConflictDetection)):
            raise NotImplementedError('ASAS drop-in: CD method %s has no device implementation '
                                      '(supported: STATEBASED, GPU)' % name)

    def _params(self, reso):
        a = self.asas
        p = _lib.SimParams(simdt=1.0, rpz=float(a.R), hpz=float(a.dh), tla=float(a.dtlookahead), cd_every=1,
                           reso=reso, mvp=mvp.params_from_asas(a), winddim=0, resume_nav=1,
                           windnorth=0.0, windeast=0.0)
        return p

    def _cd_state(self, reso, sel=slice(None)):
        """The arrays the device CD call reads (bsa_sim_update field names)."""
        t, ap = self.traf, self.traf.ap
        s = dict(lat=t.lat[sel], lon=t.lon[sel], trk=t.trk[sel], gs=t.gs[sel], alt=t.alt[sel], vs=t.vs[sel],
                 gseast=t.gseast[sel], gsnorth=t.gsnorth[sel], selalt=t.selalt[sel], ap_vs=ap.vs[sel],
                 asas_alt=np.asarray(self.asas.alt, dtype=np.float64)[sel])
        if not reso:   # DoNothing.resolve reads the autopilot targets
            s.update(ap_trk=ap.trk[sel], ap_tas=ap.tas[sel], ap_alt=ap.alt[sel])
        return s

    def _full_state(self, sel=slice(None)):
        """Every bsa_sim_state array (init / create); the kinematics-only ones are
        never read by a CD call."""
        t, ap = self.traf, self.traf.ap
        s = self._cd_state(0, sel)
        m = len(s['lat'])
        s.update(tas=getattr(t, 'tas', t.gs)[sel], hdg=getattr(t, 'hdg', t.trk)[sel])
        for k in _ZEROS:
            s[k] = np.zeros(m)
        s.update(ap_trk=ap.trk[sel], ap_tas=ap.tas[sel], ap_alt=ap.alt[sel])
        return s

    def _init(self, p, keep_counts):
        a = self.asas
        if keep_counts:
            self._base = [len(a.confpairs_all), len(a.lospairs_all)]
        else:
            self._base = [0, 0]
            self._prev_unique = (set(), set())
        if len(getattr(a, 'resopairs', ())) and not isinstance(a.resopairs, ResoPairs):
            warnings.warn('ASAS drop-in installed mid-run: the device bookkeeping starts with empty '
                          'resopairs', RuntimeWarning)
        self.ctx.sim_init(self._full_state(), p)
        self._set_ids()

    def _set_ids(self):
        self._ids = list(self.traf.id)
        self._idarr = np.asarray(self._ids, dtype=object)

    def _sync_traffic(self, p, reso):
        """Mirror Traffic.create / delete since the last call; False if the device
        sim had to be re-initialised instead."""
        ids, prev = self.traf.id, self._ids
        if len(ids) == len(prev) and list(ids) == prev:
            return True
        cur = set(ids)
        deleted = [k for k, x in enumerate(prev) if x not in cur]
        kept = [x for x in prev if x in cur]
        if list(ids[:len(kept)]) != kept or not kept:
            # not an append / delete pattern (or everything was deleted): start over
            self._init(p, keep_counts=True)
            return False
        if deleted:
            self.ctx.sim_delete(deleted)
        if len(ids) > len(kept):
            self.ctx.sim_create(self._full_state(slice(len(kept), len(ids))))
        self._set_ids()
        return True

    def _membership(self, names):
        if not names:
            return None
        s = set(names)
        return np.fromiter((i in s for i in self._ids), dtype=np.uint8, count=len(self._ids))

    # ------------------------------------------------------------- ASAS.update
    def update(self, simt):
        """ASAS.update (asas.py:473-504) with the body on the device."""
        a, traf = self.asas, self.traf
        if not a.swasas or simt < a.tasas:
            return
        a.tasas += a.dtasas
        if not traf.ntraf:
            return
        tm = [time.perf_counter()]
        self._check_cd()
        reso = self._reso_mode()
        p = self._params(reso)
        ctx = self.ctx
        if self._ids is None or a.resopairs is not self._reso:   # first call, or ASAS.reset()
            self._init(p, keep_counts=False)
        elif self._sync_traffic(p, reso):
            ctx.sim_set_params(p)
            ctx.sim_update(**self._cd_state(reso))
        noreso = self._membership(a.noresolst) if a.swnoreso else None
        resooff = self._membership(a.resoofflst) if a.swresooff else None
        if noreso is not None or resooff is not None or self._lists:
            ctx.sim_set_reso_lists(noreso, resooff)
            self._lists = noreso is not None or resooff is not None
        tm.append(time.perf_counter())
        ctx.sim_cd()
        tm.append(time.perf_counter())
        st = ctx.sim_stats()
        o = ctx.fetch_pairs(st['n_conf'], st['n_los'])
        ids = self._idarr
        a.confpairs = PairList(ids, o['ci'], o['cj'])
        a.lospairs = PairList(ids, o['li'], o['lj'])
        a.inconf = o['inconf'].astype(bool)
        a.tcpamax, a.qdr, a.dist, a.tcpa, a.tLOS = o['tcpamax'], o['qdr'], o['dist'], o['tcpa'], o['tinconf']
        tm.append(time.perf_counter())
        out = ctx.sim_read_asas()
        if len(a.confpairs):   # asas.py:486-487: the resolver ran
            if reso:
                a.trk, a.tas, a.vs, a.alt = out['trk'], out['tas'], out['vs'], out['alt']
                a.asase, a.asasn = out['asase'], out['asasn']
                if not a.asaseval:
                    a.asaseval = True
            else:              # DoNothing.resolve (DoNothing.py:11-20), the same views the reference takes
                a.trk, a.tas, a.vs, a.alt = traf.ap.trk[:], traf.ap.tas[:], traf.ap.vs[:], traf.ap.alt[:]
        a.active = out['active']
        bk = ctx.sim_asas_stats()
        a.confpairs_unique = UniquePairs(bk['confpairs_unique'], a.confpairs)
        a.lospairs_unique = UniquePairs(bk['lospairs_unique'], a.lospairs)
        if self.history:
            # the reference's own set algebra (asas.py:494-502), at the reference's cost
            cu, lu = set(a.confpairs_unique), set(a.lospairs_unique)
            if not isinstance(a.confpairs_all, list):
                a.confpairs_all, a.lospairs_all = [], []
            a.confpairs_all.extend(cu - self._prev_unique[0])
            a.lospairs_all.extend(lu - self._prev_unique[1])
            self._prev_unique = (cu, lu)
        else:
            a.confpairs_all = PairHistory(self._base[0] + bk['confpairs_all'])
            a.lospairs_all = PairHistory(self._base[1] + bk['lospairs_all'])
        a.resopairs = self._reso = ResoPairs(bk['resopairs'], self._resopairs)
        tm.append(time.perf_counter())
        if self.waypoint_recovery and out['dropped'].any():
            routes = getattr(traf.ap, 'route', None)
            if routes is not None:   # asas.py:459-462
                for i in np.flatnonzero(out['dropped']).tolist():
                    iwpid = routes[i].findact(i)
                    if iwpid != -1:
                        routes[i].direct(i, routes[i].wpname[iwpid])
        tm.append(time.perf_counter())
        self.timings = dict(upload=tm[1] - tm[0], cd=tm[2] - tm[1], pairs=tm[3] - tm[2],
                            asas_outputs=tm[4] - tm[3], waypoints=tm[5] - tm[4], total=tm[5] - tm[0])

    _lists = False

    def _resopairs(self):
        i, j = self.ctx.sim_resopairs()
        ids = self._idarr
        return {(ids[a], ids[b] if b >= 0 else None) for a, b in zip(i.tolist(), j.tolist())}


def install(asas, traf=None, ctx=None, history=False, waypoint_recovery=True):
    """Replace ``asas.update`` on this instance with the device call (the class and
    other instances are untouched).  ``traf`` defaults to ``bluesky.traf``.
    Returns the DeviceASAS (``uninstall`` restores the reference method)."""
    if traf is None:
        import bluesky as bs   # pragma: no cover
        traf = bs.traf
    dev = DeviceASAS(asas, traf, ctx=ctx, history=history, waypoint_recovery=waypoint_recovery)
    asas.update = dev.update
    return dev


def uninstall(asas):
    """Drop the instance binding: ``asas.update`` is the class's method again."""
    asas.__dict__.pop('update', None)
