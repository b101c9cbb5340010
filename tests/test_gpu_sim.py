"""GPU parity of the device-resident sim step (bsa_sim_*) against the oracle
composition of detect -> MVP -> APorASAS -> kinematics (oracle/step.py).

Every GPU step is compared with one oracle step taken from the GPU's own
previous state (re-anchored), so rounding differences cannot accumulate;
state arrays within 1e-9 relative, asas.active and conflict counts exact."""
import numpy as np
import pytest

from bluesky_amd import _lib, resident, synth
from oracle import mvp as omvp
from oracle import step as ostep
from tests import util

pytestmark = pytest.mark.gpu

SCALES = dict(lat=90.0, lon=180.0, alt=1e4, tas=300.0, hdg=360.0, vs=20.0, gs=300.0, trk=360.0,
              gseast=300.0, gsnorth=300.0, asas_trk=360.0, asas_tas=300.0, asas_vs=20.0,
              asas_alt=1e4)


PRIO_NAMES = {v: k for k, v in _lib.PRIO_CODES.items()}


def oracle_params(p, reso=True):
    return dict(simdt=p.simdt, rpz=p.rpz, hpz=p.hpz, tla=p.tla, reso=reso,
                wind=(p.windnorth, p.windeast) if p.winddim else None,
                mvp=omvp.params_from_settings(p.rpz, p.hpz, p.tla, p.mvp.Rm / p.rpz,
                                              bool(p.mvp.swresohoriz), bool(p.mvp.swresospd),
                                              bool(p.mvp.swresohdg), bool(p.mvp.swresovert),
                                              bool(p.mvp.swprio), PRIO_NAMES.get(p.mvp.priocode, 'FF1')))


def full_state(init, read):
    st = dict(init)
    for k, v in read.items():
        st[k] = v
    return st


def compare(got, exp, step):
    for k, s in SCALES.items():
        ok, msg = util.close(got[k], exp[k], s)
        assert ok, 'step %d %s: %s' % (step, k, msg)
    assert np.array_equal(got['active'], exp['active']), 'step %d active' % step


@pytest.mark.parametrize('cd_every,steps,hv,wind', [(1, 4, False, None), (3, 7, False, None),
                                                    (1, 3, True, None), (1, 4, False, (-7.5, 12.0)),
                                                    (2, 5, True, (3.0, -20.0))])
def test_resident_steps_match_oracle(ctx, cd_every, steps, hv, wind):
    t = synth.box(1500, 60.0, seed=23)
    init = resident.initial_state(t)
    p = resident.params(cd_every=cd_every, swresohoriz=not hv, wind=wind)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    op = oracle_params(p)
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(t.ntraf), active=np.zeros(t.ntraf, bool))
    for k in range(steps):
        exp = ostep.sim_step(prev, op, do_cd=(k % cd_every == 0))
        sim.step(1)
        got = full_state(init, sim.read())
        compare(got, exp, k)
        if k % cd_every == 0:
            assert sim.stats()['n_conf'] == exp['n_conf']
        prev = got
    assert sim.stats()['steps'] == steps
    assert sim.stats()['cd_calls'] == (steps + cd_every - 1) // cd_every


@pytest.mark.parametrize('prio', ['FF1', 'FF2', 'FF3', 'LAY1', 'LAY2'])
def test_resident_priority_rules_match_oracle(ctx, prio):
    """swprio with each priority code (MVP.py:235-300) on the fused path, where
    K2 evaluates MVP's per-pair vectors (k_rank, bsa_mvp_math.h) as it places
    each conflict pair; horizontal + vertical resolution so the vertical rules act."""
    t = synth.box(1500, 60.0, seed=53)
    init = resident.initial_state(t)
    rng = np.random.default_rng(53)
    init['vs'] = rng.choice([0.0, 0.0, 5.0, -7.0], t.ntraf)   # mix of level / climbing / descending
    p = resident.params(cd_every=1, swresohoriz=False, swprio=True, priocode=prio)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    op = oracle_params(p)
    assert op['mvp']['swprio'] and op['mvp']['priocode'] == prio
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(t.ntraf), active=np.zeros(t.ntraf, bool))
    for k in range(3):
        exp = ostep.sim_step(prev, op, do_cd=True)
        sim.step(1)
        got = full_state(init, sim.read())
        compare(got, exp, k)
        prev = got


def test_resident_cd_only(ctx):
    """RESO OFF, the reference's default CR (asas.py:76-77): DoNothing.resolve
    (DoNothing.py:11-20) sets the ASAS targets to the autopilot's, so active
    aircraft fly their (frozen) autopilot targets; compared with the oracle."""
    t = synth.box(800, 40.0, seed=29)
    init = resident.initial_state(t)
    p = resident.params(reso=False)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    op = oracle_params(p, reso=False)
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(t.ntraf), active=np.zeros(t.ntraf, bool))
    for k in range(2):
        exp = ostep.sim_step(prev, op, do_cd=True)
        sim.step(1)
        got = full_state(init, sim.read())
        compare(got, exp, k)
        prev = got
    assert got['active'].any()
    assert np.array_equal(got['asas_vs'][got['active']], init['ap_vs'][got['active']])
    assert np.allclose(got['hdg'], init['hdg'], rtol=0, atol=1e-9)


def test_resident_detect_matches_standalone(ctx):
    """The sim's CD on step 0 equals a standalone bsa_detect on the same state."""
    t = synth.box(3000, 150.0, seed=31)
    init = resident.initial_state(t)
    ctx.set_state(t.lat, t.lon, t.trk, t.gs, t.alt, t.vs)
    nc_ref, _ = ctx.detect(synth.RPZ, synth.HPZ, synth.TLOOKAHEAD)
    sim = resident.ResidentSim(init, resident.params(), ctx=ctx)
    sim.step(1)
    assert sim.stats()['n_conf'] == nc_ref


def test_single_rank_comm(ctx):
    """World-size-1 RCCL communicator: init, all-reduce, and a sim step through it."""
    from bluesky_amd import _lib
    c = _lib.Context(0)
    c.comm_init(1, 0, _lib.comm_unique_id())
    assert c.allreduce_max([3.0, -1.0]).tolist() == [3.0, -1.0]
    assert c.allreduce_sum([2.5]).tolist() == [2.5]
    t = synth.box(1000, 50.0, seed=37)
    init = resident.initial_state(t)
    sim = resident.ResidentSim(init, resident.params(), ctx=c)
    sim.step(2)
    ref = resident.ResidentSim(init, resident.params(), ctx=ctx)
    ref.step(2)
    a, b = sim.read(), ref.read()
    for k in SCALES:
        assert np.array_equal(a[k], b[k]), k
    c.close()


def test_resident_overflow_retry_is_exact(ctx):
    """A candidate list far too small for the traffic: every CD step overflows,
    aborts (state untouched), grows the list and re-runs.  The result must be
    bitwise the result of a run that never overflowed."""
    from bluesky_amd import _lib
    t = synth.box(2000, 80.0, seed=41)
    init = resident.initial_state(t)
    p = resident.params(cd_every=2)
    ref = resident.ResidentSim(init, p, ctx=ctx)
    ref.step(5)
    exp, exp_stats = ref.read(), ref.stats()
    c2 = _lib.Context(0)
    sim = resident.ResidentSim(init, p, ctx=c2)
    c2.set_candidate_capacity(16)
    sim.step(3)
    c2.set_candidate_capacity(16)
    sim.step(2)
    got, st = sim.read(), sim.stats()
    for k in exp:
        assert np.array_equal(got[k], exp[k]), k
    assert (st['steps'], st['cd_calls'], st['n_conf']) == (exp_stats['steps'], exp_stats['cd_calls'],
                                                          exp_stats['n_conf'])


@pytest.mark.parametrize('cd_every,steps,simdt', [(1, 8, 2.0), (2, 9, 1.5)])
def test_resident_resume_nav_matches_oracle(ctx, cd_every, steps, simdt):
    """resume_nav: device resopairs / ResumeNav / unique counts (asas.py:409-504)
    against oracle/asas.py (pinned to the reference's ASAS.update, tests/golden/
    asas_*.npz) composed into the step; resopairs compared as exact sets."""
    from oracle import asas as oasas
    t = synth.box(1500, 60.0, seed=43)
    init = resident.initial_state(t)
    p = resident.params(simdt=simdt, cd_every=cd_every, resume_nav=True)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    op = oracle_params(p)
    bk = oasas.Bookkeeping(t.ntraf)
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(t.ntraf), active=np.zeros(t.ntraf, bool))
    dropped = 0
    for k in range(steps):
        cd = k % cd_every == 0
        exp = ostep.sim_step(prev, op, do_cd=cd, bk=bk)
        sim.step(1)
        got = full_state(init, sim.read())
        compare(got, exp, k)
        if cd:
            dropped += sum(1 for v in bk.last_keep.values() if not v)
            i, j = sim.resopairs()
            assert list(zip(i.tolist(), j.tolist())) == sorted(bk.resopairs), 'step %d resopairs' % k
            st = sim.asas_stats()
            assert st == dict(resopairs=len(bk.resopairs), confpairs_unique=len(bk.confpairs_unique),
                              lospairs_unique=len(bk.lospairs_unique), confpairs_all=bk.confpairs_all,
                              lospairs_all=bk.lospairs_all, active=int(exp['active'].sum())), k
        prev = got
    assert len(bk.resopairs) > 0 and dropped > 0, (len(bk.resopairs), dropped)


def test_resident_resume_nav_overflow_retry_is_exact(ctx):
    """Resopairs buffer forced far too small mid-run: the step aborts before MVP,
    grows the buffer and re-runs; bitwise equal to an undisturbed run."""
    from bluesky_amd import _lib
    t = synth.box(2000, 80.0, seed=47)
    init = resident.initial_state(t)
    p = resident.params(simdt=1.0, resume_nav=True)
    ref = resident.ResidentSim(init, p, ctx=ctx)
    ref.step(6)
    exp, exp_bk, exp_reso = ref.read(), ref.asas_stats(), ref.resopairs()
    c2 = _lib.Context(0)
    sim = resident.ResidentSim(init, p, ctx=c2)
    sim.step(2)
    c2.set_candidate_capacity(16)   # also the resopairs capacity once bookkeeping runs
    sim.step(4)
    got, got_bk, got_reso = sim.read(), sim.asas_stats(), sim.resopairs()
    for k in exp:
        assert np.array_equal(got[k], exp[k]), k
    assert got_bk == exp_bk and exp_bk['resopairs'] > 16
    assert np.array_equal(got_reso[0], exp_reso[0]) and np.array_equal(got_reso[1], exp_reso[1])
    assert sim.stats()['steps'] == 6
    c2.close()


def test_resident_windfield_matches_oracle(ctx):
    """winddim 2: the 2-D wind field (windfield.py:158-179) read per aircraft by
    Pilot.APorASAS and UpdateGroundSpeed inside the resident step."""
    from oracle import kinematics as okin
    t = synth.box(1200, 60.0, seed=37)
    init = resident.initial_state(t)
    field = dict(lat=np.array([52.0, 52.6, 51.5, 52.3]), lon=np.array([4.0, 3.2, 4.9, 5.1]),
                 vnorth=np.array([-12.0, 3.5, 20.0, -1.0]), veast=np.array([5.0, -15.0, 2.0, 30.0]))
    p = resident.params(cd_every=1, windfield=True)
    sim = resident.ResidentSim(init, p, ctx=ctx, windfield=field)
    op = oracle_params(p)
    op['windfield'] = field
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(t.ntraf), active=np.zeros(t.ntraf, bool))
    for k in range(3):
        exp = ostep.sim_step(prev, op, do_cd=True)
        sim.step(1)
        got = full_state(init, sim.read())
        compare(got, exp, k)
        prev = got
    vn, _ = okin.windfield_2d(prev['lat'], prev['lon'], field['lat'], field['lon'], field['vnorth'],
                              field['veast'])
    assert np.ptp(vn) > 1.0      # the field actually varies over the traffic
    ctx.set_windfield()
    with pytest.raises(Exception, match='wind field'):
        sim.step(1)


def test_resident_openap_limits_match_oracle(ctx):
    """Pilot.applylimits with an OpenAP envelope (pilot.py:65-68, perfoap.py:185-209)
    between APorASAS and UpdateAirSpeed; the envelope changes the first step's
    tas of more than 10 % of the aircraft (checked below)."""
    t = synth.box(1500, 60.0, seed=41)
    init = resident.initial_state(t)
    rng = np.random.default_rng(41)
    n = t.ntraf
    init['ap_vs'] = rng.choice([0.0, 5.0, 25.0], n)
    init['ap_tas'] = init['tas'] * rng.choice([0.6, 1.0, 1.3], n)
    init['ap_alt'] = init['alt'] + rng.choice([0.0, 3000.0, -3000.0], n)
    env = dict(hmax=np.full(n, 11500.0), vmin=rng.uniform(70., 90., n), vmax=rng.uniform(140., 160., n),
               vsmin=np.full(n, -15.0), vsmax=rng.uniform(8., 12., n), axmax=np.full(n, 2.0))
    p = resident.params(cd_every=2)
    sim = resident.ResidentSim(init, p, ctx=ctx, limits=env)
    op = oracle_params(p)
    op['limits'] = env
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(n), active=np.zeros(n, bool), ax=np.zeros(n))
    for k in range(4):
        exp = ostep.sim_step(prev, op, do_cd=(k % 2 == 0))
        sim.step(1)
        got = full_state(init, sim.read())
        compare(got, exp, k)
        got['ax'] = exp['ax']      # traf.ax is device-internal; the oracle's is carried over
        prev = got
    # the envelope binds: without it the oracle's first step already differs
    free = dict(op)
    free.pop('limits')
    s0 = dict(init)
    s0.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(), asas_vs=np.zeros(n),
              active=np.zeros(n, bool), ax=np.zeros(n))
    a, b = ostep.sim_step(s0, op, do_cd=True), ostep.sim_step(s0, free, do_cd=True)
    assert np.mean(a['tas'] != b['tas']) > 0.1 and np.any(a['vs'] != b['vs'])
    ctx.sim_set_limits(None)


def test_resident_create_delete_matches_oracle(ctx):
    """Traffic.delete / create between steps (bsa_sim_delete / bsa_sim_create,
    traffic.py:192-378): every per-aircraft array is compacted / appended on the
    device and the ASAS bookkeeping follows the reference's callsign-keyed sets
    (oracle/asas.py delete / create, pinned by tests/golden/trace_super8del.npz).
    Each step is compared with the oracle step from the same state."""
    from oracle import asas as oasas
    t = synth.box(1500, 60.0, seed=83)
    init = resident.initial_state(t)
    p = resident.params(simdt=2.0, resume_nav=True)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    op = oracle_params(p)
    bk = oasas.Bookkeeping(t.ntraf)
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(t.ntraf), active=np.zeros(t.ntraf, bool))
    rng = np.random.default_rng(83)
    dangling = 0
    for k in range(9):
        if k == 3:   # delete 10 %: intruders of live resopairs among them
            i, j = sim.resopairs()
            gone = np.unique(np.concatenate([rng.choice(j, 40, replace=False),
                                             rng.choice(t.ntraf, 110, replace=False)]))
            sim.delete(gone)
            bk.delete(gone)
            keep = np.ones(len(prev['lat']), bool)
            keep[gone] = False
            init = {a: v[keep] for a, v in init.items()}
            prev = {a: v[keep] for a, v in prev.items()}
            i, j = sim.resopairs()
            dangling = int((j < 0).sum())
            assert sorted(zip(i.tolist(), j.tolist())) == sorted(bk.resopairs)
            st = full_state(init, sim.read())
            for a in SCALES:
                assert np.array_equal(st[a], prev[a]), a
            assert np.array_equal(st['active'], prev['active'])
        if k == 5:   # create 60 aircraft in the same airspace
            u = synth.box(60, 60.0, seed=84)
            new = resident.initial_state(u)
            sim.create(new)
            bk.create(60)
            init = {a: np.concatenate([init[a], new[a]]) for a in init}
            add = dict(new, asas_trk=new['trk'], asas_tas=new['tas'], asas_vs=np.zeros(60),
                       active=np.zeros(60, bool))
            prev = {a: np.concatenate([prev[a], add[a]]) for a in prev}
        exp = ostep.sim_step(prev, op, do_cd=True, bk=bk)
        sim.step(1)
        got = full_state(init, sim.read())
        compare(got, exp, k)
        i, j = sim.resopairs()
        assert list(zip(i.tolist(), j.tolist())) == sorted(bk.resopairs), 'step %d resopairs' % k
        st = sim.asas_stats()
        assert st == dict(resopairs=len(bk.resopairs), confpairs_unique=len(bk.confpairs_unique),
                          lospairs_unique=len(bk.lospairs_unique), confpairs_all=bk.confpairs_all,
                          lospairs_all=bk.lospairs_all, active=int(exp['active'].sum())), k
        assert sim.stats()['n_conf'] == exp['n_conf']
        prev = got
    assert dangling > 0 and len(got['lat']) == t.ntraf - len(gone) + 60


def test_resident_create_delete_errors(ctx):
    t = synth.box(300, 30.0, seed=89)
    init = resident.initial_state(t)
    sim = resident.ResidentSim(init, resident.params(), ctx=ctx)
    with pytest.raises(RuntimeError):
        sim.delete(np.arange(300))            # every aircraft
    with pytest.raises(RuntimeError):
        sim.delete([300])                     # out of range
    env = {k: np.full(300, v) for k, v in dict(hmax=2e4, vmin=50., vmax=300., vsmin=-20., vsmax=20.,
                                               axmax=1.).items()}
    sim.ctx.sim_set_limits(env)
    with pytest.raises(RuntimeError):
        sim.create({k: v[:2] for k, v in init.items()})   # limits on
    sim.delete([0, 0, 5])                     # duplicates ignored; limits compacted
    assert sim.ctx.n == 298 and len(sim.read()['lat']) == 298
    sim.step(1)


def test_resident_openap_phase_matches_oracle(ctx):
    """OpenAP.update in the step (bsa_sim_set_perf): flight phase from the
    pre-step vs / alt, the type x phase envelope of the reference's own
    coefficient tables (tests/golden/perf_openap3000.npz) and acceleration()
    -- against oracle/perf.py composed into the oracle step; the phase and
    traf.ax of every step exact."""
    from bluesky_amd import perf
    from tests.test_perf_oracle import load
    g, fw, rot = load()
    t = synth.box(2000, 60.0, seed=91)
    init = resident.initial_state(t)
    rng = np.random.default_rng(91)
    n = t.ntraf
    types = np.array(sorted(fw) + sorted(rot))
    actypes = types[rng.integers(0, len(types), n)]
    lifttype = np.where(np.isin(actypes, sorted(rot)), perf.LIFT_ROTOR, perf.LIFT_FIXWING)
    # ground, initial climb / approach band, climb / descent, cruise
    init['alt'] = rng.choice([0.5, 150.0, 900.0, 3000.0, 10000.0], n) + rng.uniform(-1.0, 1.0, n)
    init['vs'] = rng.choice([0.0, 0.3, -0.3, 4.0, -4.0], n)
    init['ap_alt'] = init['alt'] + rng.choice([0.0, 600.0, -600.0], n)
    init['ap_vs'] = rng.choice([2.0, 8.0, 30.0], n)
    init['ap_tas'] = init['tas'] * rng.choice([0.3, 1.0, 1.4], n)
    init['asas_alt'] = init['alt'].copy()
    # rotors never get axmax (perfoap.py:254-261): a climb above their vsmax
    # would be (1 - 0/0) * vsmax = NaN in the reference too; keep them below it
    init['ap_vs'][lifttype == perf.LIFT_ROTOR] = 2.0
    table, tidx = perf.type_table(fw, rot, actypes, lifttype)
    p = resident.params(cd_every=2)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    sim.set_perf(table, tidx)
    op = oracle_params(p)
    op['perf'] = dict(actypes=actypes, lifttype=lifttype, limits_fixwing=fw, limits_rotor=rot)
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(n), active=np.zeros(n, bool), ax=np.zeros(n))
    seen = set()
    for k in range(5):
        exp = ostep.sim_step(prev, op, do_cd=(k % 2 == 0))
        sim.step(1)
        got = full_state(init, sim.read())
        compare(got, exp, k)
        ph, ax = sim.read_perf()
        assert np.array_equal(ph, exp['phase'].astype(np.uint8)), k
        ok, msg = util.close(ax, exp['ax'], 2.0)
        assert ok, 'step %d ax: %s' % (k, msg)
        seen |= set(np.unique(ph).tolist())
        got['ax'] = ax
        prev = got
    assert {perf.NA, perf.IC, perf.CL, perf.CR, perf.DE, perf.AP, perf.GD} <= seen, seen
    sim.set_perf(None)
    with pytest.raises(RuntimeError):
        sim.set_perf(table, np.full(n, len(table), np.int32))   # index outside the table


def test_resident_row_bucket_overflow_retry_is_exact(ctx):
    """K2 row buckets one pair wide overflow on the first dense row: the
    resident step aborts, widens them and re-runs (bsa_sim_step's retry) --
    the state after several MVP steps equals the default run's bitwise."""
    from bluesky_amd import _lib
    t = synth.box(1500, 60.0, seed=53)
    init = resident.initial_state(t)
    p = resident.params(cd_every=1)
    ref = resident.ResidentSim(init, p, ctx=ctx)
    ref.step(4)
    exp = ref.read()
    c = _lib.Context(0)
    try:
        c.set_row_bucket(1)
        sim = resident.ResidentSim(init, p, ctx=c)
        sim.step(4)
        got = sim.read()
        for k in exp:
            assert np.array_equal(got[k], exp[k]), k
        assert sim.stats()['n_conf'] == ref.stats()['n_conf'] > 0
    finally:
        c.close()


def test_resident_atmosphere_outputs(ctx):
    """traf.p / rho / Temp = vatmos(traf.alt) (traffic.py:389, the first thing
    Traffic.update does, on the pre-step altitude) from the resident step when
    switched on (bsa_sim_set_atmos), against the oracle's vatmos (aero.py:62-74),
    including through a delete (the arrays follow np.delete)."""
    from oracle import kinematics as okin
    t = synth.box(3000, 150.0, seed=97)
    t.alt[:50] = np.linspace(0.0, 20000.0, 50)   # troposphere, tropopause and stratosphere
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=2), ctx=ctx)
    ctx.sim_set_atmos(True)
    for k in range(3):
        alt0 = sim.read()['alt']
        sim.step(1)
        p, rho, T = ctx.sim_read_atmos()
        ep, erho, eT = okin.vatmos(alt0)
        for g, e in ((p, ep), (rho, erho), (T, eT)):
            ok, msg = util.close(g, e, 1.0)
            assert ok, 'step %d: %s' % (k, msg)
    sim.delete([3, 7])
    p2, _, _ = ctx.sim_read_atmos()
    assert np.array_equal(p2, np.delete(p, [3, 7]))
    ctx.sim_set_atmos(False)
    with pytest.raises(_lib.AccelError):
        ctx.sim_read_atmos()


@pytest.mark.parametrize('field', ['gs', 'lat'])
def test_resident_nonfinite_aircraft(ctx, field):
    """An aircraft with a NaN state value in the resident step: the CD call's
    pairs are the finite aircraft's, every row's tcpamax is NaN as np.max makes
    it (StateBasedCD.py:90 -- the next detect's records are K4''s), and the
    step's state equals the oracle step's (NaN where the reference has NaN)."""
    t = synth.box(1500, 60.0, seed=41)
    getattr(t, field)[11] = np.nan
    init = resident.initial_state(t)
    p = resident.params(cd_every=1)
    sim = resident.ResidentSim(init, p, ctx=ctx)
    op = oracle_params(p)
    prev = dict(init)
    prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(),
                asas_vs=np.zeros(t.ntraf), active=np.zeros(t.ntraf, bool))
    for k in range(3):   # the first detect from K0b's records, the next ones from K4''s
        exp = ostep.sim_step(prev, op, do_cd=True)
        sim.step(1)
        st = sim.stats()
        assert st['n_conf'] == exp['n_conf']
        pairs = ctx.fetch_pairs(st['n_conf'], st['n_los'])
        assert np.isnan(pairs['tcpamax']).all(), 'step %d' % k
        got = full_state(init, sim.read())
        compare(got, exp, k)
        prev = got
