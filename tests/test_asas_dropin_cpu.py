"""CPU: host logic of the ASAS.update drop-in (bluesky_amd/asas.py) against a
recording stand-in for the library context -- the call cadence, how Traffic
create / delete between calls are mirrored (bsa_sim_delete / bsa_sim_create,
asas.py's callsign-keyed bookkeeping survives them), re-initialisation on
ASAS.reset(), the lazy pair containers, and that unsupported CD / CR methods
raise instead of running anywhere else."""
import types

import numpy as np
import pytest

from bluesky_amd import _lib
from bluesky_amd import asas as gasas


class RecCtx:
    """Records the Context calls the drop-in makes; returns empty results."""

    def __init__(self):
        self.calls = []
        self.n = 0

    def sim_init(self, state, p):
        self.calls.append(('init', len(state['lat'])))
        self.n = len(state['lat'])
        self.p = p

    def sim_delete(self, idx):
        self.calls.append(('delete', list(idx)))
        self.n -= len(idx)

    def sim_create(self, state):
        self.calls.append(('create', len(state['lat']), float(state['lat'][0])))
        self.n += len(state['lat'])

    def sim_set_params(self, p):
        self.calls.append(('params', p.rpz))

    def sim_update(self, **a):
        assert all(len(v) == self.n for v in a.values())
        self.calls.append(('update', sorted(a)))

    def sim_set_reso_lists(self, noreso, resooff):
        self.calls.append(('lists', None if noreso is None else noreso.tolist()))

    def sim_cd(self):
        self.calls.append(('cd',))

    def sim_stats(self):
        return dict(n_conf=0, n_los=0)

    def fetch_pairs(self, nc, nl):
        e = np.empty(0, np.int32)
        return dict(ci=e, cj=e, li=e, lj=e, inconf=np.zeros(self.n, np.uint8), tcpamax=np.zeros(self.n),
                    qdr=np.empty(0), dist=np.empty(0), tcpa=np.empty(0), tinconf=np.empty(0))

    def sim_read_asas(self):
        z = np.zeros(self.n)
        return dict(trk=z, tas=z, vs=z, alt=z, asase=z.astype(np.float32), asasn=z.astype(np.float32),
                    active=np.zeros(self.n, bool), dropped=np.zeros(self.n, bool))

    def sim_asas_stats(self):
        return dict(resopairs=0, confpairs_unique=0, lospairs_unique=0, confpairs_all=3, lospairs_all=1)

    def kinds(self):
        return [c[0] for c in self.calls]


def traffic(ids):
    n = len(ids)
    t = types.SimpleNamespace(id=list(ids), ntraf=n)
    for k in ('lat', 'lon', 'trk', 'gs', 'alt', 'vs', 'tas', 'hdg', 'gseast', 'gsnorth', 'selalt'):
        setattr(t, k, np.arange(n, dtype=np.float64))
    t.ap = types.SimpleNamespace(trk=np.zeros(n), tas=np.zeros(n), alt=np.zeros(n), vs=np.zeros(n))
    return t


def asas_obj(cr='MVP'):
    a = types.SimpleNamespace(swasas=True, tasas=0.0, dtasas=1.0, asaseval=False, noresolst=[], resoofflst=[],
                              swnoreso=False, swresooff=False, priocode='FF1', R=9260.0, dh=304.8,
                              dtlookahead=300.0, Rm=9723.0, dhm=320.0, vmin=100.0, vmax=250.0, vsmin=-15.0,
                              vsmax=15.0, swresohoriz=True, swresospd=False, swresohdg=False, swresovert=False,
                              swprio=False, resopairs=set(), confpairs_all=[], lospairs_all=[])
    a.cd = types.ModuleType('bluesky.traffic.asas.StateBasedCD')
    a.cr = types.ModuleType('bluesky.traffic.asas.' + cr)
    a.alt = np.zeros(0)
    return a


def run(a, t, simt):
    a.alt = np.zeros(t.ntraf)
    a.update(simt)


def test_create_delete_are_mirrored_and_reset_reinitialises():
    ctx = RecCtx()
    t = traffic(['A', 'B', 'C', 'D'])
    a = asas_obj()
    dev = gasas.install(a, t, ctx=ctx)
    assert a.update == dev.update
    run(a, t, 0.0)
    assert ctx.kinds() == ['init', 'cd'] and ctx.p.resume_nav == 1 and ctx.p.reso == 1
    assert ctx.p.rpz == 9260.0 and ctx.p.mvp.Rm == 9723.0
    # len() of the cumulative lists comes from the device counts
    assert len(a.confpairs_all) == 3 and len(a.lospairs_all) == 1
    with pytest.raises(RuntimeError):
        list(a.confpairs_all)
    # DEL B, D; CRE E (appended): delete of the old indices, create of the new tail
    ctx.calls.clear()
    t2 = traffic(['A', 'C', 'E'])
    t2.lat[2] = 42.0
    dev.traf = t2
    a.dtlookahead = 200.0   # DTLOOK between calls
    run(a, t2, 1.0)
    assert ctx.calls[0] == ('delete', [1, 3])
    assert ctx.calls[1] == ('create', 1, 42.0)
    assert ctx.kinds()[2:] == ['params', 'update', 'cd']
    # nothing changed: params + update only
    ctx.calls.clear()
    run(a, t2, 2.0)
    assert ctx.kinds() == ['params', 'update', 'cd']
    upd = [c for c in ctx.calls if c[0] == 'update'][0][1]
    assert 'ap_trk' not in upd and {'lat', 'gseast', 'selalt', 'ap_vs', 'asas_alt'} <= set(upd)
    # a reordering is not create / delete: re-init, the cumulative counts carry on
    ctx.calls.clear()
    dev.traf = traffic(['C', 'A', 'E'])
    run(a, dev.traf, 3.0)
    assert ctx.kinds() == ['init', 'cd'] and len(a.confpairs_all) == 6
    # ASAS.reset(): a fresh resopairs set -> re-init with counts from zero
    ctx.calls.clear()
    a.resopairs, a.confpairs_all, a.lospairs_all = set(), [], []
    run(a, dev.traf, 4.0)
    assert ctx.kinds() == ['init', 'cd'] and len(a.confpairs_all) == 3
    # cadence
    ctx.calls.clear()
    run(a, dev.traf, 4.5)
    assert ctx.calls == []
    gasas.uninstall(a)
    assert 'update' not in a.__dict__


def test_cr_off_uploads_autopilot_targets_and_lists_reach_the_device():
    ctx = RecCtx()
    t = traffic(['A', 'B', 'C'])
    a = asas_obj('DoNothing')
    gasas.install(a, t, ctx=ctx)
    run(a, t, 0.0)
    assert ctx.p.reso == 0
    run(a, t, 1.0)
    upd = [c for c in ctx.calls if c[0] == 'update'][-1][1]
    assert {'ap_trk', 'ap_tas', 'ap_alt'} <= set(upd)
    a.swnoreso, a.noresolst = True, ['B']
    run(a, t, 2.0)
    assert ('lists', [0, 1, 0]) in ctx.calls
    ctx.calls.clear()
    a.swnoreso = False
    run(a, t, 3.0)
    assert ('lists', None) in ctx.calls     # cleared once on the device
    ctx.calls.clear()
    run(a, t, 4.0)
    assert 'lists' not in ctx.kinds()


@pytest.mark.parametrize('what', ['cd', 'cr'])
def test_unsupported_methods_raise(what):
    a = asas_obj()
    if what == 'cd':
        a.cd = types.ModuleType('bluesky.traffic.asas.casas')
    else:
        a.cr = types.ModuleType('bluesky.traffic.asas.SSD')
    t = traffic(['A'])
    gasas.install(a, t, ctx=RecCtx())
    with pytest.raises(NotImplementedError):
        run(a, t, 0.0)


def test_lazy_pair_containers():
    ids = np.asarray(['A', 'B', 'C'], dtype=object)
    pl = gasas.PairList(ids, np.array([0, 1, 2]), np.array([1, 0, 1]))
    assert len(pl) == 3 and bool(pl) and pl._list is None
    assert pl[0] == ('A', 'B') and list(pl) == [('A', 'B'), ('B', 'A'), ('C', 'B')]
    assert pl == [('A', 'B'), ('B', 'A'), ('C', 'B')]
    assert not gasas.PairList(ids, np.empty(0, int), np.empty(0, int))
    u = gasas.UniquePairs(2, pl)
    assert len(u) == 2 and frozenset(('A', 'B')) in u and set(u) == {frozenset('AB'), frozenset('BC')}
    assert u - {frozenset('AB')} == {frozenset('BC')}
    r = gasas.ResoPairs(1, lambda: {('A', None)})
    assert len(r) == 1 and ('A', None) in r


def test_no_context_means_no_compute():
    """Without a HIP device the drop-in cannot be created (no CPU path)."""
    lib = _lib.load()
    if lib.bsa_device_count() > 0:
        pytest.skip('a HIP device is visible here')
    with pytest.raises(_lib.AccelUnavailable):
        gasas.install(asas_obj(), traffic(['A']))


def test_several_ranks_are_refused():
    """a context joined to a communicator holds only its rows'
    outputs (and no global counts): the drop-in refuses it up front."""
    ctx = RecCtx()
    ctx.comm_rank_world = (1, 2)
    with pytest.raises(NotImplementedError, match='one rank only'):
        gasas.install(asas_obj(), traffic(['A', 'B']), ctx=ctx)


class Route:
    """ap.route[i] stand-in: records Route.direct calls (asas.py:459-462)."""

    def __init__(self, log, act):
        self.log, self.act, self.wpname = log, act, ['WP0', 'WP1', 'WP2']

    def findact(self, i):
        return self.act

    def direct(self, i, name):
        self.log.append((i, name))


def test_waypoint_recovery_follows_the_device_drop_flags():
    """ResumeNav's waypoint recovery (asas.py:459-462): route.direct to the
    active waypoint for exactly the aircraft whose pair the device dropped
    (bsa_sim_read_asas `dropped`, aircraft-index order), none without an active
    waypoint, nothing with waypoint_recovery=False."""
    class DropCtx(RecCtx):
        def sim_read_asas(self):
            o = super().sim_read_asas()
            o['dropped'] = np.array([False, True, False, True, True])
            return o

    log = []
    t = traffic(['A', 'B', 'C', 'D', 'E'])
    t.ap.route = [Route(log, 1), Route(log, 2), Route(log, 0), Route(log, -1), Route(log, 0)]
    a = asas_obj()
    gasas.install(a, t, ctx=DropCtx())
    run(a, t, 0.0)
    assert log == [(1, 'WP2'), (4, 'WP0')]
    log.clear()
    a2 = asas_obj()
    gasas.install(a2, t, ctx=DropCtx(), waypoint_recovery=False)
    run(a2, t, 0.0)
    assert log == []
