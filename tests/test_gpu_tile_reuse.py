"""Tile-pair list reuse of the resident step: K0d's item
list is built on boxes grown by the drift budgets and kept while every
aircraft's prefilter record stays inside them (K4' checks; the first record
outside makes the next detect rebuild on the device).  It only changes which
detects rebuild the coarse cull -- every pair is still tested and evaluated --
so the sim with it is BITWISE the sim without it: state arrays and pair lists
after every step, with MVP manoeuvres, large steps that force rebuilds, budgets
tiny enough to rebuild every step, and cd_every > 1."""
import numpy as np
import pytest

from bluesky_amd import _lib, resident, synth

pytestmark = pytest.mark.gpu


def run(ctx, init, p, steps, tile):
    if tile is None:
        ctx.set_tile_reuse(False)
    else:
        ctx.set_tile_reuse(True, *tile)
    try:
        sim = resident.ResidentSim(init, p, ctx=ctx)
        out = []
        for _ in range(steps):
            sim.step(1)
            st = sim.stats()
            out.append((sim.read(), ctx.fetch_pairs(st['n_conf'], st['n_los'])))
        return out, ctx.tile_reuse_stats()
    finally:
        ctx.set_tile_reuse(True)


def same(a, b):
    for k, (sa, pa) in enumerate(a):
        sb, pb = b[k]
        for f in sa:
            assert np.array_equal(sa[f], sb[f]), 'step %d %s' % (k, f)
        for f in ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'li', 'lj', 'inconf', 'tcpamax'):
            assert np.array_equal(pa[f], pb[f]), 'step %d %s' % (k, f)


@pytest.mark.parametrize('simdt, tile, cd_every', [
    (0.05, (2016.0, 300.0), 1),     # the bench's cadence and default budgets: few builds
    (1.0, (2016.0, 300.0), 1),      # 250 m per step: rebuilds every few steps
    (1.0, (1.0, 1.0), 1),           # budgets below one step's drift: a rebuild at every detect
    (0.5, (2016.0, 300.0), 3),      # K4' prepares (and checks) only before CD steps
])
def test_tile_reuse_is_bitwise_the_full_cull(ctx, simdt, tile, cd_every):
    t = synth.box(20000, 300.0, seed=101)
    init = resident.initial_state(t)
    p = resident.params(simdt=simdt, cd_every=cd_every, swresohoriz=False)   # horizontal + vertical MVP
    exp, _ = run(ctx, init, p, 24, None)
    got, st = run(ctx, init, p, 24, tile)
    same(got, exp)
    assert sum(len(x[1]['ci']) for x in exp) > 0
    assert st['builds'] >= 1


def test_tile_reuse_builds_rarely_at_the_bench_cadence(ctx):
    """At simdt 0.05 s the list survives many detects (the point of keeping
    it), and a budget below one step's drift rebuilds every time."""
    t = synth.box(20000, 300.0, seed=103)
    init = resident.initial_state(t)
    p = resident.params(simdt=0.05)
    _, a0 = run(ctx, init, p, 0, (2016.0, 300.0))
    _, a = run(ctx, init, p, 30, (2016.0, 300.0))
    builds, detects = a['builds'] - a0['builds'], a['detects'] - a0['detects']
    # (the first detect is K0b's: no list; HK rebuilds at 0.75 of the budgets, and the first
    # steps of the sim are its vertical transient -- aircraft levelling off -- so a few more)
    assert detects == 29 and 1 <= builds <= 12, a
    _, b0 = run(ctx, init, resident.params(simdt=1.0), 0, (1.0, 1.0))
    h0 = ctx.hk_stats()
    _, b = run(ctx, init, resident.params(simdt=1.0), 10, (1.0, 1.0))
    # (HK: the host keeps the list right after a build; that step finds it stale and
    # re-runs without a list -- the re-run counts no list detect -- then the device
    # decides for a while: a rebuild at every other detect)
    stale = ctx.hk_stats()['stale_aborts'] - h0['stale_aborts']
    assert b['builds'] - b0['builds'] == b['detects'] - b0['detects'] == 9 - stale, (b, stale)


@pytest.mark.parametrize('us', ['0', '20', '1e9'])
def test_longest_items_first_is_bitwise(monkeypatch, us):
    """The prefilter's listed items ("longest items first"):
    the slots whose units took longer than the threshold at the last detect
    are swept first and skipped among the regular units.  Threshold 0 lists
    every slot (each is swept once, as a listed item), 1e9 none: the state and
    the pair lists are bitwise those of a run without tile-pair list reuse."""
    monkeypatch.setenv('BSA_PF_HEAVY_US', us)
    c = _lib.Context(0)
    try:
        t = synth.box(20000, 300.0, seed=109)
        init = resident.initial_state(t)
        p = resident.params(simdt=0.5, swresohoriz=False)
        exp, _ = run(c, init, p, 12, None)
        got, st = run(c, init, p, 12, (2016.0, 300.0))
        same(got, exp)
        assert sum(len(x[1]['ci']) for x in exp) > 0
        assert st['detects'] >= 9   # (11 list detects, less an HK-kept one gone stale and re-run without a list)
    finally:
        c.close()


# ---------------------------------------------------------------- host-known decisions (HK)
def run_batch(ctx, init, p, batches, hk, f=0.75):
    """The resident sim in batches of steps (one bsa_sim_step call each, so the
    host enqueues ahead of the device and waits on the published predictions),
    with HK on / off; the state and pair lists after every batch."""
    ctx.set_hk(hk, f)
    try:
        sim = resident.ResidentSim(init, p, ctx=ctx)
        h0 = ctx.hk_stats()
        out = []
        for k in batches:
            sim.step(k)
            st = sim.stats()
            out.append((sim.read(), ctx.fetch_pairs(st['n_conf'], st['n_los'])))
        h = ctx.hk_stats()
        return out, {k: h[k] - h0[k] for k in ('keeps', 'builds', 'waits', 'stale_aborts')}
    finally:
        ctx.set_hk(True, 0.75)


@pytest.mark.parametrize('simdt, f, horiz', [
    (0.05, 0.75, True),    # the bench's cadence and MVP: kept lists, the host waits on the predictions
    (0.05, 0.75, False),   # vertical MVP: vs jumps move the midpoint altitudes (budget 300 m) at once
    (1.0, 0.75, False),    # 250 m per step: predicted rebuilds every few detects
    (1.0, 4.0, False),     # predictions far too late: kept lists go stale, their steps re-run rebuilt
])
def test_host_known_decisions_are_bitwise(ctx, simdt, f, horiz):
    """HK: the host decides each detect's rebuild before it
    enqueues the detect, from a prediction the device published two detects
    earlier; a kept detect launches no K0d.  A kept list that no longer covers
    the records aborts its step (Counters::tpr_stale), which re-runs with a
    build.  Neither changes a result: bitwise the device-decided run."""
    t = synth.box(20000, 300.0, seed=113)
    init = resident.initial_state(t)
    p = resident.params(simdt=simdt, swresohoriz=horiz)
    batches = [1, 5, 30, 1, 20]
    exp, h_off = run_batch(ctx, init, p, batches, False)
    got, h = run_batch(ctx, init, p, batches, True, f)
    same(got, exp)
    assert h_off['keeps'] == h_off['builds'] == 0
    assert sum(len(x[1]['ci']) for x in exp) > 0
    assert h['keeps'] > 0 and h['builds'] >= 1, h
    if f > 1.0:
        assert h['stale_aborts'] >= 1, h
    elif horiz:   # (no vertical MVP jumps: the predictions come in time -- the first steps' levelling-off
        assert h['stale_aborts'] == 0 and h['keeps'] > h['builds'], h   # transient still rebuilds often)
