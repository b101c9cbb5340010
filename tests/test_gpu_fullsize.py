"""GPU parity at the BASELINE sizes (configs[2] box10k, configs[3] box100k,
configs[4] global 1M) -- the cases the golden fixtures are too small for.

* box10k: the whole detect against the oracle (10^8 pairs, ~15-30 s of CPU).
* box100k: the whole detect against the oracle's (10^10 pairs, evaluated on
  the CPU of the build container by tools/make_fullrows.py into a fixture).
* Exact-safety of the culling at full size: the pruned detect (fp32 stage 1 +
  CPA refine) must equal the unpruned one
  (BSA_FLAG_NOPRUNE: every pair of the rows evaluated in fp64), bitwise, for
  EVERY row at 100k (row slabs, StateBasedCD.py:82-101 for all 10^10 pairs)
  and EVERY row at 1M global (10^12 pairs, eight tests of 256-row slabs, incl.
  the |lat| > 60 deg rows).
* global 1M: the full detect's structure (row-major order, inconf <=> rows with
  pairs, tcpamax >= 0) plus 32 rows against the oracle over all 1M columns.
* the resident step at 100k: five re-anchored steps of MVP + pilot +
  kinematics against the oracle composition fed with the GPU's pair lists of
  the same state (verified per step).
"""
import numpy as np
import pytest

from bluesky_amd import _lib, resident, statebased, synth
from oracle import statebased as ocd
from oracle import step as ostep
from tests import util

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
RPZ, HPZ, TLA = synth.RPZ, synth.HPZ, synth.TLOOKAHEAD
FIELDS = ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'dcpa', 'li', 'lj', 'inconf', 'tcpamax')


def _bitwise_rows(full, part, rb, re):
    """part (rows [rb, re) of a detect) == the same rows of full, bitwise."""
    sel = (full['ci'] >= rb) & (full['ci'] < re)
    lsel = (full['li'] >= rb) & (full['li'] < re)
    for k in FIELDS:
        if k in ('li', 'lj'):
            exp = full[k][lsel]
        elif k in ('inconf', 'tcpamax'):
            exp = full[k][rb:re]
        else:
            exp = full[k][sel]
        got = part[k]
        assert got.shape == exp.shape, '%s rows [%d, %d): %s != %s' % (k, rb, re, got.shape, exp.shape)
        assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(exp).view(np.uint8)), \
            '%s rows [%d, %d) differ' % (k, rb, re)


def test_box10k_full_vs_oracle(ctx):
    """BASELINE configs[2]: 10k aircraft in a 500 NM box, the whole pair set."""
    t = synth.workload('box10k')
    got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
    exp = ocd.detect_arrays(t, t, RPZ, HPZ, TLA, budget_bytes=1 << 30)
    util.assert_detect_equal(got, exp, RPZ, TLA)
    # the survey's probe count for this recipe at seed 7
    assert (len(got['ci']), len(got['li'])) == (14317, 2228)


def test_box100k_every_row_vs_oracle_fixture(ctx):
    """BASELINE configs[3] against the ORACLE over every row:
    tests/golden/full_box100k.npz holds the oracle's StateBasedCD.detect of the
    whole 100k box (1e10 pairs, evaluated on the CPU by tools/make_fullrows.py):
    the HIP detect's conflict / LoS pair lists equal it pair for pair and in
    order, inconf exactly, and qdr / dist / tcpa / tinconf / dcpa / tcpamax
    within 1e-9 relative (tests/util.py)."""
    import hashlib
    path = util.golden('full_box100k.npz')
    assert path, 'tests/golden/full_box100k.npz missing (python tools/make_fullrows.py)'
    z = dict(np.load(path[0], allow_pickle=False))
    t = synth.workload('box100k')
    h = hashlib.sha256()
    for f in ('lat', 'lon', 'trk', 'gs', 'alt', 'vs'):
        h.update(np.ascontiguousarray(getattr(t, f), dtype=np.float64).tobytes())
    assert h.hexdigest() == str(z['state_sha256']), 'the synthetic box100k differs from the fixture\'s'
    got = statebased.detect_indices(t, t, float(z['rpz']), float(z['hpz']), float(z['tla']), ctx=ctx,
                                    with_dcpa=True)
    n = int(z['n'])
    inconf = np.unpackbits(z['inconf_bits'])[:n].astype(bool)
    tcpamax = np.zeros(n)
    tcpamax[inconf] = z['tcpamax_inconf']
    exp = dict(ci=z['ci'], cj=z['cj'], li=z['li'], lj=z['lj'], qdr=z['qdr'], dist=z['dist'], tcpa=z['tcpa'],
               tinconf=z['tinconf'], inconf=inconf, tcpamax=tcpamax)
    util.assert_detect_equal(got, exp, RPZ, TLA)
    ok, msg = util.close(got['dcpa'], z['dcpa'], RPZ)
    assert ok, 'dcpa: %s' % msg
    assert len(exp['ci']) > 100000 and len(exp['li']) > 10000


def test_noprune_row_sweep_100k_bitwise(ctx):
    """Every row of the 100k box: pruned detect == unpruned detect, bitwise."""
    t = synth.workload('box100k')
    n = t.ntraf
    full = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx, with_dcpa=True)
    slab = 2048
    flags = _lib.FLAG_NOPRUNE | _lib.FLAG_WITH_DCPA
    for rb in range(0, n, slab):
        re = min(n, rb + slab)
        nc, nl = ctx.detect(RPZ, HPZ, TLA, flags, rb, re)
        part = ctx.fetch_pairs(nc, nl, with_dcpa=True)
        _bitwise_rows(full, part, rb, re)
    assert len(full['ci']) > 100000


def test_global1m_structure_and_oracle_rows(ctx):
    """BASELINE configs[4] (1M global) on one GPU: properties of the full
    detect and 32 rows against the oracle over all 1M columns."""
    t = synth.workload('global1m')
    n = t.ntraf
    got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
    key = got['ci'].astype(np.int64) * n + got['cj']
    assert len(key) > 10000 and np.all(np.diff(key) > 0)
    lkey = got['li'].astype(np.int64) * n + got['lj']
    assert np.all(np.diff(lkey) > 0)
    assert np.array_equal(np.unique(got['ci']), np.flatnonzero(got['inconf']))
    assert np.all(got['tcpamax'] >= 0) and np.all(got['tcpamax'][~got['inconf'].astype(bool)] == 0)
    assert np.all(got['ci'] != got['cj']) and np.all(got['tinconf'] < TLA)
    rng = np.random.default_rng(5)
    hi = np.flatnonzero(np.abs(t.lat) > 60.0)
    rows = np.unique(np.concatenate([rng.choice(n, 24, replace=False), rng.choice(hi, 8, replace=False),
                                     got['ci'][rng.choice(len(got['ci']), 8, replace=False)]]))
    exp = ocd.detect_arrays(t, t, RPZ, HPZ, TLA, rows=rows, budget_bytes=512 << 20)
    sel = np.isin(got['ci'], rows)
    lsel = np.isin(got['li'], rows)
    sub = dict(ci=got['ci'][sel], cj=got['cj'][sel], li=got['li'][lsel], lj=got['lj'][lsel],
               qdr=got['qdr'][sel], dist=got['dist'][sel], tcpa=got['tcpa'][sel],
               tinconf=got['tinconf'][sel], inconf=got['inconf'][rows], tcpamax=got['tcpamax'][rows])
    util.assert_detect_equal(sub, exp, RPZ, TLA)


_G1M = {}


def _global1m_full(ctx):
    """The pruned detect of the whole 1M set, computed once for the sweep parts."""
    if 'full' not in _G1M:
        t = synth.workload('global1m')
        _G1M['t'] = t
        _G1M['full'] = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx, with_dcpa=True)
    return _G1M['t'], _G1M['full']


def _bitwise_rows_sorted(full, part, rb, re):
    """_bitwise_rows for row-major sorted ``full`` (row slices by binary search)."""
    c0, c1 = np.searchsorted(full['ci'], [rb, re])
    l0, l1 = np.searchsorted(full['li'], [rb, re])
    for k in FIELDS:
        if k in ('li', 'lj'):
            exp = full[k][l0:l1]
        elif k in ('inconf', 'tcpamax'):
            exp = full[k][rb:re]
        else:
            exp = full[k][c0:c1]
        got = part[k]
        assert got.shape == exp.shape, '%s rows [%d, %d): %s != %s' % (k, rb, re, got.shape, exp.shape)
        assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(exp).view(np.uint8)), \
            '%s rows [%d, %d) differ' % (k, rb, re)


@pytest.mark.parametrize('part', range(8))
def test_noprune_row_sweep_global1m_bitwise(ctx, part):
    """EVERY row of the 1M global set (BASELINE configs[4]), one eighth per
    test: pruned detect == unpruned detect (every pair of the slab's rows
    evaluated in fp64, StateBasedCD.py:82-101), bitwise, in 256-row slabs
    (2.6e8 pairs each).  The eight parts cover rows 0..1M exactly once."""
    t, full = _global1m_full(ctx)
    n = t.ntraf
    flags = _lib.FLAG_NOPRUNE | _lib.FLAG_WITH_DCPA
    per = (n + 7) // 8
    slab = 256
    lo, hi = part * per, min(n, (part + 1) * per)
    high = 0
    for rb in range(lo, hi, slab):
        re = min(hi, rb + slab)
        nc, nl = ctx.detect(RPZ, HPZ, TLA, flags, rb, re)
        _bitwise_rows_sorted(full, ctx.fetch_pairs(nc, nl, with_dcpa=True), rb, re)
        high += int(np.sum(np.abs(t.lat[rb:re]) > 60.0))
    assert high > 100       # every eighth holds rows in the |lat| > 60 deg bands


def test_resident_steps_100k_vs_oracle(ctx):
    """Five consecutive resident steps (CD + MVP + pilot + kinematics) at the
    bench size, each against the oracle composition (oracle/step.py) started
    from the GPU's previous state (re-anchored): every state array incl. MVP's
    persistent asas.alt (MVP.py:128-143) <= 1e-9, asas.active exact.  The N^2
    oracle detect is out of reach at 100k, so each step's pair lists come from
    a standalone GPU detect of the same state, checked per step: the sim's
    conflict count, 4096 rows pruned == unpruned bitwise, 8 rows against the
    oracle over all 100k columns."""
    from tests.test_gpu_sim import SCALES, oracle_params
    t = synth.workload('box100k')
    n = t.ntraf
    init = resident.initial_state(t)
    p = resident.params(cd_every=1)
    op = oracle_params(p)
    c2 = _lib.Context(0)
    try:
        sim = resident.ResidentSim(init, p, ctx=ctx)
        prev = dict(init)
        prev.update(asas_trk=init['trk'].copy(), asas_tas=init['tas'].copy(), asas_vs=np.zeros(n),
                    active=np.zeros(n, bool))
        rng = np.random.default_rng(11)
        flags = _lib.FLAG_NOPRUNE | _lib.FLAG_WITH_DCPA
        for k in range(5):
            cur = synth.Traffic(prev['lat'], prev['lon'], prev['alt'], prev['trk'], prev['gs'], prev['vs'])
            cd = statebased.detect_indices(cur, cur, RPZ, HPZ, TLA, ctx=c2, with_dcpa=True)
            for rb in rng.choice(n // 2048, 2, replace=False) * 2048:
                nc, nl = c2.detect(RPZ, HPZ, TLA, flags, int(rb), int(rb) + 2048)
                _bitwise_rows(cd, c2.fetch_pairs(nc, nl, with_dcpa=True), int(rb), int(rb) + 2048)
            rows = np.unique(np.concatenate([rng.choice(n, 4, replace=False),
                                             cd['ci'][rng.choice(len(cd['ci']), 4, replace=False)]]))
            exp_rows = ocd.detect_arrays(cur, cur, RPZ, HPZ, TLA, rows=rows, budget_bytes=256 << 20)
            sel, lsel = np.isin(cd['ci'], rows), np.isin(cd['li'], rows)
            sub = {f: cd[f][sel] for f in ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf')}
            sub.update(li=cd['li'][lsel], lj=cd['lj'][lsel], inconf=cd['inconf'][rows],
                       tcpamax=cd['tcpamax'][rows])
            util.assert_detect_equal(sub, exp_rows, RPZ, TLA)
            exp = ostep.sim_step(prev, op, do_cd=True, cd=cd)
            sim.step(1)
            assert sim.stats()['n_conf'] == len(cd['ci']) == exp['n_conf'], k
            got = dict(init)
            got.update(sim.read())
            for f, sc in SCALES.items():
                ok, msg = util.close(got[f], exp[f], sc)
                assert ok, 'step %d %s: %s' % (k, f, msg)
            assert np.array_equal(got['active'], exp['active']), k
            prev = got
    finally:
        c2.close()
