"""The nranks > 1 paths of libbsaccel on ONE GPU: several
contexts in one process form the ranks of the row-sharded resident sim through
the in-process group transport (bsa_group_*, bsa_comm.hip), one host thread per
rank.  Everything the RCCL path does between ranks runs here too -- the state
all-gather before each CD (k_pack / k_unpack), the gate all-reduce, the global
unique-pair key all-gather, the C2 rank-order pair gather -- only the transport
differs (device-to-device copies instead of xGMI).

The sharded run must equal the one-rank run BITWISE: rows are independent in
detect, MVP and the kinematics, so rank 0 (+) rank 1 (+) ... is the same
arithmetic on the same inputs.
"""
import threading

import numpy as np
import pytest

from bluesky_amd import _lib, dist, resident, statebased, synth

pytestmark = pytest.mark.gpu
RPZ, HPZ, TLA = synth.RPZ, synth.HPZ, synth.TLOOKAHEAD


def run_ranks(world, fn, timeout=240):
    """fn(rank, ctx, group) on `world` threads, each with its own context."""
    group = _lib.Group(world)
    ctxs = [_lib.Context(0) for _ in range(world)]
    out, err = [None] * world, [None] * world

    def body(r):
        try:
            out[r] = fn(r, ctxs[r], group)
        except BaseException as e:   # noqa: BLE001 -- reported below
            err[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    alive = [t.is_alive() for t in th]
    if not any(alive):
        for c in ctxs:
            c.close()
        group.close()
    assert not any(alive), 'rank threads hung'
    errs = [e for e in err if e is not None]
    if errs:   # a rank's own failure, not the barrier timeout it left the others in
        first = [e for e in errs if 'barrier' not in str(e)] or errs
        raise AssertionError('rank errors: %s' % ['%d: %r' % (r, e) for r, e in enumerate(err) if e]) from first[0]
    return out


def world1(init, p, steps, ctx):
    sim = resident.ResidentSim(init, p, ctx=ctx)
    sim.step(steps)
    return sim


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_resident_steps_equal_world1(ctx, world):
    """10 steps with MVP (CD every step): every state array of the sharded run
    equals the one-rank run bitwise, and the C2 pair gather of the last CD call
    equals the one-rank pair lists."""
    t = synth.box(3001, 100.0, seed=61)
    init = resident.initial_state(t)
    p = resident.params(cd_every=1, swresohoriz=False)   # horizontal + vertical MVP
    ref = world1(init, p, 10, ctx)
    exp, exp_st = ref.read(), ref.stats()
    exp_pairs = ctx.fetch_pairs(exp_st['n_conf'], exp_st['n_los'])

    def rank(r, c, g):
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=world, group=g)
        sim.step(4)
        sim.step(6)
        return sim.read(), sim.stats(), sim.gather_pairs(root=0)

    res = run_ranks(world, rank)
    for r, (got, st, pairs) in enumerate(res):
        for k in exp:
            assert np.array_equal(got[k], exp[k]), 'rank %d %s' % (r, k)
        assert st['steps'] == 10 and st['cd_calls'] == 10
    n_conf = sum(st['n_conf'] for _, st, _ in res)
    assert n_conf == exp_st['n_conf'] > 0
    pairs = res[0][2]
    assert all(x[2] is None for x in res[1:])
    for k in ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'li', 'lj', 'inconf', 'tcpamax'):
        assert np.array_equal(pairs[k], exp_pairs[k]), k


def test_sharded_resume_nav_global_counts_equal_world1(ctx):
    """resume_nav: resopairs (union over ranks), asas.active and the GLOBAL
    unique / cumulative pair counts (asas.py:490-502, all-gathered key blocks)
    equal the one-rank run at every CD call."""
    t = synth.box(2500, 70.0, seed=67)
    init = resident.initial_state(t)
    p = resident.params(simdt=1.0, resume_nav=True)
    ref = resident.ResidentSim(init, p, ctx=ctx)
    exp = []
    for _ in range(6):
        ref.step(1)
        i, j = ref.resopairs()
        exp.append((ref.asas_stats(), sorted(zip(i.tolist(), j.tolist())), ref.read()['active']))

    def rank(r, c, g):
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=2, group=g)
        got = []
        for _ in range(6):
            sim.step(1)
            i, j = sim.resopairs()
            got.append((sim.asas_stats(), list(zip(i.tolist(), j.tolist())), sim.read()['active']))
        return got

    res = run_ranks(2, rank)
    for k in range(6):
        est, ereso, eact = exp[k]
        reso = sorted(res[0][k][1] + res[1][k][1])
        assert reso == ereso, k
        for r in range(2):
            st = res[r][k][0]
            for f in ('confpairs_unique', 'lospairs_unique', 'confpairs_all', 'lospairs_all'):
                assert st[f] == est[f], (k, r, f)
            assert np.array_equal(res[r][k][2], eact), k
        assert res[0][k][0]['resopairs'] + res[1][k][0]['resopairs'] == est['resopairs']
    assert exp[-1][0]['confpairs_all'] > exp[0][0]['confpairs_unique'] > 0


def test_sharded_overflow_on_one_rank_is_exact(ctx):
    """A candidate list far too small on rank 1 only: rank 1 overflows, the gate
    all-reduce aborts the step on BOTH ranks, rank 1 grows its list while rank 0
    re-runs with unchanged buffers (bsa_sim_step); the same for a resopairs
    overflow.  The result is bitwise the undisturbed one-rank run's."""
    t = synth.box(2000, 80.0, seed=71)
    init = resident.initial_state(t)
    p = resident.params(simdt=1.0, resume_nav=True, cd_every=2)
    ref = world1(init, p, 7, ctx)
    exp, exp_bk = ref.read(), ref.asas_stats()

    def rank(r, c, g):
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=2, group=g)
        sim.step(2)
        if r == 1:
            c.set_candidate_capacity(16)    # also the resopairs capacity once bookkeeping runs
        sim.step(5)
        return sim.read(), sim.asas_stats(), sim.stats()

    res = run_ranks(2, rank)
    for r, (got, bk, st) in enumerate(res):
        for k in exp:
            assert np.array_equal(got[k], exp[k]), 'rank %d %s' % (r, k)
        for f in ('confpairs_unique', 'lospairs_unique', 'confpairs_all', 'lospairs_all'):
            assert bk[f] == exp_bk[f], (r, f)
        assert st['steps'] == 7


@pytest.mark.slow
def test_sharded_100k_key_blocks_regrow(ctx):
    """At the bench size each rank's pair keys exceed the initial all-gather
    block (65536 words): the step aborts, the blocks regrow (keeping the
    previous call's sets) and the counts still equal the one-rank run's."""
    t = synth.workload('box100k')
    init = resident.initial_state(t)
    p = resident.params(resume_nav=True)
    ref = resident.ResidentSim(init, p, ctx=ctx)
    exp = []
    for _ in range(3):
        ref.step(1)
        exp.append(ref.asas_stats())

    def rank(r, c, g):
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=2, group=g)
        got = []
        for _ in range(3):
            sim.step(1)
            got.append(sim.asas_stats())
        return got

    res = run_ranks(2, rank)
    for k in range(3):
        for r in range(2):
            for f in ('confpairs_unique', 'lospairs_unique', 'confpairs_all', 'lospairs_all'):
                assert res[r][k][f] == exp[k][f], (k, r, f)
    assert exp[0]['confpairs_unique'] > 65536


def test_sharded_standalone_detect_gather(ctx):
    """bsa_detect on each rank's row slice, then the C2 gather to rank 1: the
    8-tuple's arrays of the whole set, in the reference's row-major order."""
    t = synth.global_traffic(20000, seed=73)
    full = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx, with_dcpa=True)

    def rank(r, c, g):
        c.comm_init_group(g, r)
        rb, re = [(0, 7000), (7000, 7001), (7001, 20000)][r]
        statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=c, row_begin=rb, row_end=re, with_dcpa=True)
        return c.gather_pairs(root=1, with_dcpa=True)

    res = run_ranks(3, rank)
    assert res[0] is None and res[2] is None
    for k in full:
        assert np.array_equal(res[1][k], full[k]), k


def test_home_ranges_and_row_ids(ctx):
    """Home order: the ranks' home ranges are 512-aligned and
    tile 0..n, their aircraft (bsa_sim_row_ids) partition the indices, and each
    rank's share of a CD step (bsa_sim_detect_rows on one GPU) gives exactly
    the rows of the whole detect."""
    t = synth.box(3001, 100.0, seed=67)
    init = resident.initial_state(t)
    p = resident.params(cd_every=1)
    world = 3

    def rank(r, c, g):
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=world, group=g)
        return sim.stats(), sim.row_ids()

    res = run_ranks(world, rank)
    edges = [(st['row_begin'], st['row_end']) for st, _ in res]
    assert edges[0][0] == 0 and edges[-1][1] == t.ntraf
    assert all(a[1] == b[0] for a, b in zip(edges, edges[1:]))
    assert all(rb % 512 == 0 for rb, _ in edges)
    assert edges == [dist.home_range(t.ntraf, r, world) for r in range(world)]   # the host formula
    assert all(len(i) == re - rb for (rb, re), (_, i) in zip(edges, res))
    ids = np.concatenate([i for _, i in res])
    assert np.array_equal(np.sort(ids), np.arange(t.ntraf))
    assert all(np.all(np.diff(i) > 0) for _, i in res)
    # one GPU: the sim's detect of each rank's home slice vs the full detect
    full = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
    c = _lib.Context(0)
    try:
        sim = resident.ResidentSim(init, p, ctx=c)
        parts = []
        for (rb, re), (_, rid) in zip(edges, res):
            nc, nl = c.sim_detect_rows(rb, re)
            got = c.fetch_pairs(nc, nl)
            parts.append(got)
            sel = np.isin(full['ci'], rid)
            assert np.array_equal(got['ci'], full['ci'][sel]) and np.array_equal(got['cj'], full['cj'][sel])
            assert np.array_equal(got['qdr'], full['qdr'][sel])
            lsel = np.isin(full['li'], rid)
            assert np.array_equal(got['li'], full['li'][lsel])
            assert np.array_equal(got['inconf'], full['inconf'][rid])
            assert np.array_equal(got['tcpamax'], full['tcpamax'][rid])
        # the host merge of the ranks' shares (rows interleave in index order)
        merged = dist.merge_rank_pairs(parts, rows=[rid for _, rid in res])
        for k in ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'li', 'lj', 'inconf', 'tcpamax'):
            assert np.array_equal(merged[k], full[k]), k
        assert sim.stats()['steps'] == 0
    finally:
        c.close()


# ---------------------------------------------------------------- halo exchange
def sharded_vs_world1(ctx, t, p, world, steps, between=None, resume_nav=False, tile=None):
    """World-1 run vs ``world`` in-process ranks: every state array bitwise, the
    C2-gathered pair lists bitwise (and the ASAS bookkeeping with resume_nav)
    after each of ``steps`` steps; ``between(k, sim)`` may change parameters
    before step k on every rank; ``tile`` = tile-pair list reuse budgets of
    every run (None: the one-rank run rebuilds at every detect, the ranks use
    the defaults).  Returns the ranks' halo statistics (with each rank's
    tile_reuse_stats in the last step's) and the one-rank results."""
    init = resident.initial_state(t)
    if tile is None:
        ctx.set_tile_reuse(False)
    else:
        ctx.set_tile_reuse(True, *tile)
    try:
        ref = resident.ResidentSim(init, p, ctx=ctx)
        t0 = ctx.tile_reuse_stats()
        exp = []
        for k in range(steps):
            if between:
                between(k, ref)
            ref.step(1)
            st = ref.stats()
            e = dict(state=ref.read(), pairs=ctx.fetch_pairs(st['n_conf'], st['n_los']))
            if resume_nav:
                i, j = ref.resopairs()
                e.update(bk=ref.asas_stats(), reso=sorted(zip(i.tolist(), j.tolist())))
            exp.append(e)
        exp[-1]['tile'] = {k: v - t0[k] for k, v in ctx.tile_reuse_stats().items()}
    finally:
        ctx.set_tile_reuse(True)

    def rank(r, c, g):
        if tile is not None:
            c.set_tile_reuse(True, *tile)
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=world, group=g)
        got = []
        for k in range(steps):
            if between:
                between(k, sim)
            sim.step(1)
            e = dict(state=sim.read(), pairs=sim.gather_pairs(root=0), halo=sim.halo_stats())
            if resume_nav:
                i, j = sim.resopairs()
                e.update(bk=sim.asas_stats(), reso=list(zip(i.tolist(), j.tolist())))
            got.append(e)
        got[-1]['halo'] = dict(got[-1]['halo'], tile=c.tile_reuse_stats())
        return got

    res = run_ranks(world, rank, timeout=600)
    for k in range(steps):
        for r in range(world):
            g = res[r][k]
            for f, v in exp[k]['state'].items():
                assert np.array_equal(g['state'][f], v), 'step %d rank %d %s' % (k, r, f)
        pairs = res[0][k]['pairs']
        for f in ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'li', 'lj', 'inconf', 'tcpamax'):
            assert np.array_equal(pairs[f], exp[k]['pairs'][f]), 'step %d %s' % (k, f)
        if resume_nav:
            assert sorted(sum((res[r][k]['reso'] for r in range(world)), [])) == exp[k]['reso'], k
            for r in range(world):
                for f in ('confpairs_unique', 'lospairs_unique', 'confpairs_all', 'lospairs_all'):
                    assert res[r][k]['bk'][f] == exp[k]['bk'][f], (k, r, f)
    return [[res[r][k]['halo'] for k in range(steps)] for r in range(world)], exp


@pytest.mark.slow
def test_halo_8ranks_global1m_equal_world1(ctx):
    """BASELINE configs[4]: 1M aircraft on the globe, ownship rows over 8 ranks
    (in-process group on one GPU: the same halo plan, pack / exchange / unpack
    as over RCCL).  5 steps with MVP (CD every step): every state array and the
    gathered pair lists bitwise equal to the one-rank run after every step; each
    rank receives far less than the full state (48 MB per CD call at 1M)."""
    t = synth.workload('global1m')
    halo, exp = sharded_vs_world1(ctx, t, resident.params(cd_every=1), 8, 5)
    assert len(exp[-1]['pairs']['ci']) > 0
    rx = [h[-1]['rx_bytes'] for h in halo]
    assert max(rx) < 10 * 2 ** 20, rx           # verdict r02: <= 10 MB per rank per CD step
    assert all(h[-1]['tiles'] > 0 for h in halo)
    assert all(h[-1]['regrowths'] == 0 for h in halo)   # exact initial capacities


def test_halo_requests_and_regrowth_equal_world1(ctx):
    """ResumeNav reads the state of every resopair's intruder, wherever it is:
    after conflicts found with a long look-ahead, DTLOOK drops to 20 s, so the
    box test no longer reaches many kept resopairs' intruders -- they come in
    through the request bits.  Then ZONER grows the zone: the halo outgrows its
    capacities, the step aborts, every rank regrows the same capacities and
    re-runs.  Bitwise equal to the one-rank run throughout (state, pairs,
    resopairs, global counts)."""
    t = synth.box(20000, 800.0, seed=83)
    p0 = resident.params(simdt=5.0, tla=300.0, resume_nav=True)
    p1 = resident.params(simdt=5.0, tla=20.0, resume_nav=True)
    p2 = resident.params(simdt=5.0, tla=900.0, rpz=40 * resident.NM, resume_nav=True)

    def between(k, sim):
        if k == 3:
            sim.set_params(p1)
        if k == 6:
            sim.set_params(p2)

    halo, exp = sharded_vs_world1(ctx, t, p0, 3, 9, between=between, resume_nav=True)
    assert exp[5]['bk']['resopairs'] > 0
    assert max(h[-1]['regrowths'] for h in halo) > 0


def test_halo_wind_then_calm_equal_world1(ctx):
    """with wind K4' computes gs / trk FROM gseast / gsnorth
    (traffic.py:463-466), so a receiver may not rebuild gseast / gsnorth as
    gs sin / cos(trk).  Steps with a constant wind, then set_params without
    wind: the first calm exchange must still carry all 8 fields (only rows K4'
    wrote without wind are derivable), and the run stays bitwise equal to the
    one-rank run (state, gathered pair lists) at every step."""
    t = synth.box(3000, 100.0, seed=97)
    windy = resident.params(simdt=1.0, wind=(9.0, -14.0))
    calm = resident.params(simdt=1.0)

    def between(k, sim):
        if k == 3:
            sim.set_params(calm)

    halo, exp = sharded_vs_world1(ctx, t, windy, 2, 6, between=between)
    assert len(exp[3]['pairs']['ci']) > 0
    # 8 fields per halo row up to the first calm CD call (its state is still
    # K4' with wind), 6 from the next one on (rx_bytes: the capacities' regions)
    for h in halo:
        if h[4]['rx_bytes'] and h[3]['regrowths'] == h[4]['regrowths']:
            assert h[3]['rx_bytes'] > h[4]['rx_bytes'] == h[5]['rx_bytes'], h


@pytest.mark.parametrize('world, simdt, tile, steps, swh', [
    (3, 0.05, (2016.0, 300.0), 30, True),    # the bench cadence: plan + list kept over many detects
    (3, 0.05, (2016.0, 300.0), 16, False),   # + vertical MVP: vs changes move the records' intervals
    (2, 1.0, (2016.0, 300.0), 16, True),     # 250 m per step: some record leaves its box often
    (3, 1.0, (1.0, 1.0), 8, True),           # budgets below one step's drift: rebuild at every detect
])
def test_halo_plan_reuse_equal_world1(ctx, world, simdt, tile, steps, swh):
    """DESIGN.md 3.18 across ranks: the halo plan, the send / receive lists and
    K0d's tile-pair list are built on grown boxes and kept while every rank's
    records stay inside them (each rank's own-tile K0b raises a flag that
    travels with the box all-gather; one raised flag rebuilds all three on
    every rank).  Bitwise equal to the one-rank run after every step, with MVP
    manoeuvres.  Every rank decides alike, and about as often as the one-rank
    run with the same budgets (whose K4' checks the same records: the ranks
    also rebuild when the halo's fields change, 8 -> 6 after the first K4')."""
    t = synth.box(20000, 300.0, seed=103)
    p = resident.params(simdt=simdt, swresohoriz=swh)
    halo, exp = sharded_vs_world1(ctx, t, p, world, steps, tile=tile)
    assert sum(len(e['pairs']['ci']) for e in exp) > 0
    st = [h[-1]['tile'] for h in halo]
    assert len({(s['builds'], s['detects']) for s in st}) == 1, st   # every rank decides alike
    b, d = st[0]['builds'], st[0]['detects']
    b1 = exp[-1]['tile']['builds']
    print('world %d simdt %g swh %s: builds %d of %d detects (one rank: %d of %d)' %
          (world, simdt, swh, b, d, b1, exp[-1]['tile']['detects']))
    assert steps <= d <= steps + 2, st      # (+ a re-run step after a capacity regrowth)
    if tile == (1.0, 1.0):
        assert b == d, st
    else:
        assert 1 <= b <= b1 + 3, (st, exp[-1]['tile'])
        if swh and simdt == 0.05:
            assert b <= 8, st


@pytest.mark.parametrize('world, f', [(3, 0.75), (3, 4.0), (8, 0.75)])
def test_halo_host_known_decisions_equal_world1(ctx, world, f):
    """HK at several ranks: a kept plan skips the box
    all-gather, the halo plan and K0d on every rank alike and prepares own +
    halo tiles in one K0b; predictions travel with the gate all-reduce; a stale
    kept list on one rank re-runs the step on all (f = 4: predictions too late).
    Batches of steps, so every rank's host runs ahead of its device.  Bitwise
    the one-rank run."""
    t = synth.box(12000, 200.0, seed=127)
    init = resident.initial_state(t)
    p = resident.params(simdt=1.0, swresohoriz=False)
    batches = [1, 6, 12]

    def steps(sim):
        out = []
        for k in batches:
            sim.step(k)
            out.append(sim.read())
        return out

    exp = steps(resident.ResidentSim(init, p, ctx=ctx))

    def rank(r, c, g):
        c.set_hk(True, f)
        got = steps(resident.ResidentSim(init, p, ctx=c, rank=r, world=world, group=g))
        return got, c.hk_stats()

    res = run_ranks(world, rank)
    for r, (got, h) in enumerate(res):
        for k, st in enumerate(exp):
            for fld, v in st.items():
                assert np.array_equal(got[k][fld], v), 'rank %d batch %d %s' % (r, k, fld)
    hs = [h for _, h in res]
    assert all(h == hs[0] or (h['keeps'], h['builds']) == (hs[0]['keeps'], hs[0]['builds']) for h in hs), hs
    assert hs[0]['keeps'] > 0, hs
    if f > 1.0:
        assert hs[0]['stale_aborts'] >= 1, hs


@pytest.mark.parametrize('world', [3, 8])
def test_halo_overlap_equal_world1(ctx, world):
    """on a kept-plan detect each rank sends / receives
    its halo, prepares the received tiles and sweeps their items on a second
    stream while its own tiles are prepared and swept (bsa_set_halo_overlap 1;
    off by default), joined before K1b.  Bitwise the one-rank run, and every rank
    overlapped the same detects; with the overlap off, none."""
    t = synth.box(12000, 200.0, seed=131)
    init = resident.initial_state(t)
    p = resident.params(simdt=1.0, swresohoriz=False)
    batches = [1, 6, 12]

    def steps(sim):
        out = []
        for k in batches:
            sim.step(k)
            out.append(sim.read())
        return out

    exp = steps(resident.ResidentSim(init, p, ctx=ctx))
    for mode in (1, 0):
        def rank(r, c, g):
            c.set_halo_overlap(mode)
            got = steps(resident.ResidentSim(init, p, ctx=c, rank=r, world=world, group=g))
            return got, c.halo_overlap_count(), c.hk_stats()

        res = run_ranks(world, rank)
        for r, (got, _, _) in enumerate(res):
            for k, st in enumerate(exp):
                for fld, v in st.items():
                    assert np.array_equal(got[k][fld], v), 'mode %d rank %d batch %d %s' % (mode, r, k, fld)
        counts = [n for _, n, _ in res]
        if mode:
            assert counts[0] > 0 and counts == [counts[0]] * world, (counts, res[0][2])
        else:
            assert counts == [0] * world, counts


def test_probe_overlap_is_bitwise():
    """The halo overlap in the one-GPU probe (mode 2, tools/probe_step.py's
    measurement of its cost): one rank's share stepped with and without it
    ends in the same state bit for bit."""
    t = synth.box(20000, 200.0, seed=137)
    init = resident.initial_state(t)
    out = []
    for mode in (2, 0):
        c = _lib.Context(0)
        try:
            c.set_halo_overlap(mode)
            sim = resident.ResidentSim(init, resident.params(cd_every=1), ctx=c)
            c.sim_probe_rank(2, 4)
            sim.step(1)
            sim.step(20)
            out.append((sim.read(), c.halo_overlap_count()))
            c.sim_probe_rank(0, 1)
        finally:
            c.close()
    (a, na), (b, nb) = out
    assert na > 0 and nb == 0, (na, nb)
    for fld, v in a.items():
        assert np.array_equal(v, b[fld]), fld


def test_halo_capacity_disagreement_fails_loudly():
    """RCCL's grouped send / recv hangs or truncates when a send
    length differs from its receive length, which only 8 GPUs would show.  The
    in-process group checks every (sender, receiver) region length against the
    receiver's expectation at each exchange: one rank with a different copy of
    one tile capacity fails loudly on one GPU, and its peer does not hang."""
    t = synth.box(3000, 100.0, seed=97)
    init = resident.initial_state(t)
    p = resident.params(simdt=1.0)

    def rank(r, c, g):
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=2, group=g)
        sim.step(1)
        if r == 1:
            c.sim_set_halo_cap(0, 1, 0)
        sim.step(1)

    # (the collective layout check of the next exchange may catch it first: the
    # field count changes from 8 to 6 after the first calm K4', a new layout)
    with pytest.raises(AssertionError, match='halo (exchange|lengths disagree): rank 0 sends'):
        run_ranks(2, rank, timeout=200)


def test_halo_layout_check_is_collective():
    """VERDICT r04 missing #2: the layout check that guards the RCCL branch
    (halo_check_layout, bsa_comm.hip) runs on every rank after bsa_sim_init
    and every regrowth, before any grouped send / recv is enqueued, through the
    same host all-reduce RCCL uses: a disagreeing capacity copy on one rank
    fails the step on BOTH ranks with the same message (no rank waits in a
    send that has no matching receive)."""
    t = synth.box(3000, 100.0, seed=97)
    init = resident.initial_state(t)
    p = resident.params(simdt=1.0)

    def rank(r, c, g):
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=2, group=g)
        sim.step(1)
        if r == 1:
            c.sim_set_halo_cap(0, 1, 0)
        c.sim_halo_recheck()
        try:
            sim.step(1)
        except _lib.AccelError as e:
            return str(e)
        return None

    res = run_ranks(2, rank, timeout=200)
    assert all(m is not None and 'halo lengths disagree: rank 0 sends' in m for m in res), res


def test_halo_probe_shares_equal_full_detect(ctx):
    """bsa_sim_detect_rows as one rank of 8 computes its share (own tiles, halo
    plan, halo tiles only) at the 100k bench workload: the 8 shares' pairs
    together are exactly the full detect's (same pairs, same payload bits), and
    each share needs only part of the other ranks' tiles."""
    t = synth.workload('box100k')
    n = t.ntraf
    c2 = _lib.Context(0)
    try:
        full = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=c2)
    finally:
        c2.close()
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx)
    rpr = ((n + 7) // 8 + 511) // 512 * 512
    nct = (n + 511) // 512
    parts = []
    for r in range(8):
        rb, re = r * rpr, min(n, (r + 1) * rpr)
        nc, nl = ctx.sim_detect_rows(rb, re)
        parts.append(ctx.fetch_pairs(nc, nl))
        tiles = ctx.sim_halo_stats()['tiles']
        assert 0 < tiles < nct - (re - rb + 511) // 512, (r, tiles)
    for a, b, pay in (('ci', 'cj', ('qdr', 'dist', 'tcpa', 'tinconf')), ('li', 'lj', ())):
        i = np.concatenate([p[a] for p in parts])
        j = np.concatenate([p[b] for p in parts])
        o = np.lexsort((j, i))
        assert np.array_equal(i[o], full[a]) and np.array_equal(j[o], full[b]), a
        for f in pay:
            assert np.array_equal(np.concatenate([p[f] for p in parts])[o], full[f]), f
    assert sum(int(p['inconf'].sum()) for p in parts) == int(full['inconf'].sum())
    assert sim.stats()['steps'] == 0


def test_halo_probe_shares_nonfinite_column_outside_halo(ctx):
    """a rank's share (bsa_sim_detect_rows, halo mode) equals the
    whole detect also when the one non-finite column is outside the share's
    halo: tcpamax = max_j(tcpa * swconfl) is NaN on EVERY row
    (StateBasedCD.py:90), whichever tiles the share holds."""
    t = synth.box(20000, 1000.0, seed=73)
    t.gs[5] = np.nan
    n, R = t.ntraf, 8
    c2 = _lib.Context(0)
    try:
        full = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=c2)
    finally:
        c2.close()
    assert np.isnan(full['tcpamax']).all() and len(full['ci']) > 0
    resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx)
    rpr = ((n + R - 1) // R + 511) // 512 * 512
    nct = (n + 511) // 512
    parts, partial = [], 0
    for r in range(R):
        rb, re = r * rpr, min(n, (r + 1) * rpr)
        nc, nl = ctx.sim_detect_rows(rb, re)
        got = ctx.fetch_pairs(nc, nl)
        parts.append(got)
        assert np.isnan(got['tcpamax']).all(), r
        partial += ctx.sim_halo_stats()['tiles'] < nct - (re - rb + 511) // 512
    assert partial >= R // 2     # most shares hold part of the tiles: the NaN column is outside some halos
    i = np.concatenate([p['ci'] for p in parts])
    j = np.concatenate([p['cj'] for p in parts])
    o = np.lexsort((j, i))
    assert np.array_equal(i[o], full['ci']) and np.array_equal(j[o], full['cj'])


# ---------------------------------------------------------------- create / delete while sharded
def test_sharded_create_delete_equal_world1(ctx):
    """Traffic.delete / create during a sharded run (traffic.py:192-378,
    trafficarrays.py:73-118): 3 ranks delete 10 % of the aircraft -- intruders
    of live resopairs among them, so dangling pairs cross ranks -- and later
    create 90; the home ranges are re-partitioned and the bookkeeping rows move
    with their aircraft.  State, pair lists, resopairs and the global counts
    stay bitwise equal to the one-rank run at every step."""
    t = synth.box(3000, 100.0, seed=89)
    p = resident.params(simdt=2.0, resume_nav=True)
    rng = np.random.default_rng(89)
    new = resident.initial_state(synth.box(90, 100.0, seed=90))
    plan = {}

    def between(k, sim):
        if k == 3:
            if 'gone' not in plan:     # the one-rank run goes first: intruders of its resopairs
                _, j = sim.resopairs()
                plan['gone'] = np.unique(np.concatenate([rng.choice(j, min(40, len(j)), replace=False),
                                                         rng.choice(t.ntraf, 260, replace=False)]))
            sim.delete(plan['gone'])
        if k == 5:
            sim.create(new)

    halo, exp = sharded_vs_world1(ctx, t, p, 3, 9, between=between, resume_nav=True)
    assert len(exp[-1]['state']['lat']) == t.ntraf - len(plan['gone']) + 90
    assert exp[3]['bk']['resopairs'] > 0


def test_sharded_trace_super8del_equal_world1(ctx):
    """The reference's own DEL / CRE trace (tests/golden/trace_super8del.npz)
    replayed through the resident step at world 2 equals world 1 bitwise:
    state, resopairs, the four counts and asas.active after every call."""
    from tests import util
    from tests.test_gpu_trace import sim_state
    from tests.test_oracle_trace import traffic_change
    st, calls = util.load_trace(util.golden('trace_super8del.npz')[0])
    p = resident.params(rpz=float(st['rpz']), hpz=float(st['hpz']), tla=float(st['tla']), mar=float(st['mar']),
                        reso=True, swresohoriz=bool(st['swresohoriz']), swresospd=bool(st['swresospd']),
                        swresohdg=bool(st['swresohdg']), swresovert=bool(st['swresovert']),
                        resume_nav=True, simdt=0.05)

    def replay(sim):
        out = []
        for c, r in enumerate(calls):
            n = len(r['lat'])
            if c and 'ids' in r:
                deleted, created = traffic_change(calls[c - 1]['ids'], r['ids'])
                if deleted:
                    sim.delete(deleted)
                if created:
                    sim.create(sim_state(r, slice(n - created, n)))
            sim.update(lat=r['lat'], lon=r['lon'], trk=r['trk'], gs=r['gs'], alt=r['alt'], vs=r['vs'],
                       tas=r['tas'], gseast=r['gseast'], gsnorth=r['gsnorth'], selalt=r['selalt'],
                       ap_vs=r['apvs'], ap_trk=r['aptrk'], ap_tas=r['aptas'], ap_alt=r['apalt'])
            sim.step(1)
            i, j = sim.resopairs()
            out.append((sim.read(), sim.asas_stats(), list(zip(i.tolist(), j.tolist()))))
        return out

    init = sim_state(calls[0], slice(None))
    exp = replay(resident.ResidentSim(init, p, ctx=ctx))
    res = run_ranks(2, lambda r, c, g: replay(resident.ResidentSim(init, p, ctx=c, rank=r, world=2, group=g)))
    for k, (est, ebk, ereso) in enumerate(exp):
        for f, v in est.items():
            for r in range(2):
                assert np.array_equal(res[r][k][0][f], v), 'call %d rank %d %s' % (k, r, f)
        assert sorted(res[0][k][2] + res[1][k][2]) == sorted(ereso), k
        for r in range(2):
            for f in ('confpairs_unique', 'lospairs_unique', 'confpairs_all', 'lospairs_all'):
                assert res[r][k][1][f] == ebk[f], (k, r, f)
    assert any(len(x[2]) for x in exp)


@pytest.mark.parametrize('world', [2, 3])
def test_bench_parity_vs_world1_group(world):
    """bench.py's self-check at world > 1, through the
    in-process group on one GPU: the sharded steps' all-gathered state and
    gathered pairs equal rank 0's own world-1 run, every rank gets ok."""
    import bench
    t = synth.box(3001, 100.0, seed=61)
    init = resident.initial_state(t)
    p = resident.params(cd_every=1)

    def rank(r, c, g):
        return bench.parity_vs_world1(c, init, p, r, world, 0, steps=2, group=g)

    res = run_ranks(world, rank)
    assert all(x['ok'] for x in res), res
    assert res[0]['mismatched'] == [] and res[0]['n_conf'] > 0 and len(res[0]['state_sha256']) == 64


def test_probe_rank_step_runs_one_rank_share():
    """bsa_sim_probe_rank (measurement aid of tools/probe_step.py): a one-rank
    sim steps only rank r's home rows in the one-GPU halo mode; the rows of the
    other ranks do not move, and nranks = 1 returns to the whole sim."""
    t = synth.box(3001, 100.0, seed=61)
    init = resident.initial_state(t)
    c = _lib.Context(0)
    try:
        sim = resident.ResidentSim(init, resident.params(cd_every=1), ctx=c)
        before = sim.read()
        c.sim_probe_rank(1, 2)
        sim.step(3)
        st = sim.stats()
        assert (st['row_begin'], st['row_end']) == dist.home_range(t.ntraf, 1, 2)
        after = sim.read()
        mine = np.zeros(t.ntraf, bool)
        mine[sim.row_ids()] = True
        assert not np.array_equal(after['lat'][mine], before['lat'][mine])   # its rows moved
        assert np.array_equal(after['lat'][~mine], before['lat'][~mine])     # the others did not
        c.sim_probe_rank(0, 1)
        assert (sim.stats()['row_begin'], sim.stats()['row_end']) == (0, t.ntraf)
    finally:
        c.close()


def test_sharded_nonfinite_aircraft_equal_world1(ctx):
    """A NaN ground speed on one aircraft (one rank's row): every rank's
    tcpamax is NaN (the gate's non-finite word, all-reduced), as at world 1,
    and the sharded state equals the one-rank state (NaN where it is NaN)."""
    t = synth.box(3001, 100.0, seed=67)
    t.gs[1234] = np.nan
    init = resident.initial_state(t)
    p = resident.params(cd_every=1)
    ref = world1(init, p, 3, ctx)
    exp, exp_st = ref.read(), ref.stats()
    exp_pairs = ctx.fetch_pairs(exp_st['n_conf'], exp_st['n_los'])
    assert np.isnan(exp_pairs['tcpamax']).all()

    def rank(r, c, g):
        sim = resident.ResidentSim(init, p, ctx=c, rank=r, world=2, group=g)
        sim.step(3)
        return sim.read(), sim.gather_pairs(root=0)

    res = run_ranks(2, rank)
    for r, (got, _) in enumerate(res):
        for k in exp:
            assert np.array_equal(got[k], exp[k], equal_nan=got[k].dtype.kind == 'f'), 'rank %d %s' % (r, k)
    pairs = res[0][1]
    for k in ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'li', 'lj', 'inconf'):
        assert np.array_equal(pairs[k], exp_pairs[k]), k
    assert np.isnan(pairs['tcpamax']).all()
