"""Candidate-list reuse (bsa_set_candidate_reuse): a list
built with inflated reaches is re-evaluated while every aircraft stays inside
its drift budgets.  The results must be bitwise those of full detects, on the
host detect path (arbitrary state sequences) and in the resident step."""
import numpy as np
import pytest

from bluesky_amd import _lib, resident, statebased, synth

pytestmark = pytest.mark.gpu

RPZ, HPZ, TLA = synth.RPZ, synth.HPZ, synth.TLOOKAHEAD


def advance(t, dt, rng, turn_deg=0.0, dvs=0.0, dgs=0.0):
    """Straight-line motion over dt plus optional random heading / vs / gs changes."""
    R = 6371000.0
    trk = np.radians(t.trk)
    lat = t.lat + np.degrees(t.gs * np.cos(trk) * dt / R)
    lon = t.lon + np.degrees(t.gs * np.sin(trk) * dt / (R * np.cos(np.radians(t.lat))))
    alt = t.alt + t.vs * dt
    ntrk = (t.trk + turn_deg * rng.standard_normal(t.ntraf)) % 360.0
    nvs = t.vs + dvs * rng.standard_normal(t.ntraf) * (t.vs != 0)
    ngs = t.gs + dgs * rng.standard_normal(t.ntraf)
    return synth.Traffic(lat, lon, alt, ntrk, ngs, nvs)


def same(a, b, where):
    for k in a:
        if a[k] is None:
            continue
        assert np.array_equal(a[k], b[k]), '%s: %s differs' % (where, k)


@pytest.mark.parametrize('sh,sv', [(800.0, 60.0), (200.0, 5.0)])
def test_host_detect_reuse_is_exact(ctx, sh, sv):
    """A sequence of small steps, maneuvers and one large jump: every detect
    of the reusing context equals a fresh full detect; the list is reused."""
    rng = np.random.default_rng(3)
    t = synth.box(6000, 150.0, seed=5)
    a = _lib.Context(0)
    a.set_candidate_reuse(True, sh, sv)
    plan = [(0.05, 0, 0, 0)] * 6 + [(0.05, 0.3, 0.02, 0.05)] * 6 + [(30.0, 0, 0, 0)] + [(0.05, 0, 0, 0)] * 4
    for k, (dt, turn, dvs, dgs) in enumerate(plan):
        got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, with_dcpa=True, ctx=a)
        exp = statebased.detect_indices(t, t, RPZ, HPZ, TLA, with_dcpa=True, ctx=ctx)
        same(got, exp, 'detect %d' % k)
        t = advance(t, dt, rng, turn, dvs, dgs)
    st = a.reuse_stats()
    assert st['detects'] == len(plan)
    assert 2 <= st['builds'] < st['detects'], st
    a.close()


def test_host_reuse_invalidated_by_parameters_and_rows(ctx):
    """Changing RPZ / tla / the row range / n forces a build; results exact."""
    t = synth.box(3000, 100.0, seed=9)
    a = _lib.Context(0)
    a.set_candidate_reuse(True, 800.0, 60.0)
    for rpz, tla in ((RPZ, TLA), (RPZ, TLA), (RPZ * 1.5, TLA), (RPZ, 120.0), (RPZ, TLA)):
        got = statebased.detect_indices(t, t, rpz, HPZ, tla, ctx=a)
        exp = statebased.detect_indices(t, t, rpz, HPZ, tla, ctx=ctx)
        same(got, exp, 'rpz %g tla %g' % (rpz, tla))
    # a row slice cannot reuse (records are not shared); the next full call rebuilds
    got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=a, row_begin=100, row_end=2000)
    exp = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx, row_begin=100, row_end=2000)
    same(got, exp, 'slice')
    t2 = synth.box(2500, 100.0, seed=10)
    for tt in (t, t2, t2):
        same(statebased.detect_indices(tt, tt, RPZ, HPZ, TLA, ctx=a),
             statebased.detect_indices(tt, tt, RPZ, HPZ, TLA, ctx=ctx), 'n=%d' % tt.ntraf)
    st = a.reuse_stats()
    # builds: first, rpz, tla, back to defaults, the slice (never reuses), after
    # the slice, new n -- and the two repeats reuse
    assert st['builds'] == 7 and st['detects'] == 9, st
    a.close()


def test_host_reuse_with_overflow(ctx):
    """A too-small candidate list on a reused context: retry rebuilds, exact."""
    rng = np.random.default_rng(4)
    t = synth.box(4000, 120.0, seed=12)
    a = _lib.Context(0)
    a.set_candidate_reuse(True, 800.0, 60.0)
    for k in range(4):
        if k == 2:
            a.set_candidate_capacity(64)
        same(statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=a),
             statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx), 'detect %d' % k)
        t = advance(t, 0.05, rng)
    a.close()


@pytest.mark.parametrize('simdt,steps,resume_nav,sh,sv', [(0.05, 40, False, 800.0, 60.0),
                                                         (0.05, 24, False, 1500.0, 300.0),
                                                         (1.0, 12, True, 4000.0, 600.0)])
def test_resident_reuse_is_exact(ctx, simdt, steps, resume_nav, sh, sv):
    """The resident step with reuse is bitwise the resident step without."""
    t = synth.box(20000, 300.0, seed=17)
    init = resident.initial_state(t)
    p = resident.params(simdt=simdt, resume_nav=resume_nav)
    ref = resident.ResidentSim(init, p, ctx=_lib.Context(0))
    c2 = _lib.Context(0)
    c2.set_candidate_reuse(True, sh, sv)
    sim = resident.ResidentSim(init, p, ctx=c2)
    for k in range(steps // 4):
        ref.step(4)
        sim.step(4)
        a, b = sim.read(), ref.read()
        for key in a:
            assert np.array_equal(a[key], b[key]), 'step %d %s' % (4 * (k + 1), key)
        assert sim.stats() == ref.stats()
        if resume_nav:
            assert sim.asas_stats() == ref.asas_stats()
    st = c2.reuse_stats()
    assert st['builds'] < st['detects'], st
    print('reuse', simdt, st)
    c2.close()
    ref.ctx.close()
