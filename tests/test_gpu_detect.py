"""GPU parity: bsa_detect (HIP, gfx950) against the reference's golden vectors
and the oracle restatement; exact pair sets, reals within 1e-9 relative."""
import numpy as np
import pytest

from bluesky_amd import statebased, synth
from oracle import statebased as ocd
from tests import util

pytestmark = pytest.mark.gpu

CD = util.golden('cd_*.npz')
KWIK = util.golden('cdkwik_*.npz')
RPZ, HPZ, TLA = synth.RPZ, synth.HPZ, synth.TLOOKAHEAD


@pytest.mark.parametrize('path', CD, ids=[util.case_name(p) for p in CD])
def test_detect_matches_reference_golden(ctx, path):
    own, intr, z = util.load_cd(path)
    got = statebased.detect_indices(own, intr, float(z['rpz']), float(z['hpz']), float(z['tla']), ctx=ctx)
    util.assert_detect_equal(got, z, float(z['rpz']), float(z['tla']))


@pytest.mark.parametrize('path', CD, ids=[util.case_name(p) for p in CD])
def test_prefilter_is_exact_safe_on_golden(ctx, path):
    """Pruned (midpoint and t = 0 stage 1) and unpruned (every pair evaluated)
    runs give identical results."""
    own, intr, z = util.load_cd(path)
    a = statebased.detect_indices(own, intr, float(z['rpz']), float(z['hpz']), float(z['tla']), ctx=ctx)
    b = statebased.detect_indices(own, intr, float(z['rpz']), float(z['hpz']), float(z['tla']),
                                  ctx=ctx, noprune=True)
    c = statebased.detect_indices(own, intr, float(z['rpz']), float(z['hpz']), float(z['tla']),
                                  ctx=ctx, stage1_t0=True)
    for k in a:
        if a[k] is not None:
            nan = a[k].dtype.kind == 'f'   # (tcpamax of the non-finite cases)
            assert np.array_equal(a[k], b[k], equal_nan=nan), k
            assert np.array_equal(a[k], c[k], equal_nan=nan), k


def test_midpoint_stage1_stress_sets_vs_oracle(ctx):
    """Fast high-latitude traffic, long look-ahead, a big zone, own != intruder
    (tests/test_stage1_bound.py checks the bound itself on the same sets)."""
    from tests.test_stage1_bound import _stress_sets
    for name, own, intr, rpz, hpz, tla in _stress_sets():
        got = statebased.detect_indices(own, intr, rpz, hpz, tla, ctx=ctx)
        exp = ocd.detect_arrays(own, intr, rpz, hpz, tla)
        util.assert_detect_equal(got, exp, rpz, tla)


def test_tuple_contract(ctx):
    own, intr, z = util.load_cd(util.golden('cd_box500.npz')[0])
    res = statebased.detect(own, own, RPZ, HPZ, TLA)
    assert len(res) == 8
    confpairs, lospairs, inconf, tcpamax, qdr, dist, tcpa, tin = res
    assert isinstance(confpairs, list) and isinstance(confpairs[0], tuple)
    assert confpairs == [(own.id[i], own.id[j]) for i, j in zip(z['ci'], z['cj'])]
    assert lospairs == [(own.id[i], own.id[j]) for i, j in zip(z['li'], z['lj'])]
    assert inconf.dtype == bool and inconf.shape == (own.ntraf,)
    res9 = statebased.detect(own, own, RPZ, HPZ, TLA, with_dcpa=True)
    assert len(res9) == 9 and len(res9[6]) == len(confpairs)
    ref = ocd.detect_arrays(own, own, RPZ, HPZ, TLA, want_dcpa=True)
    ok, msg = util.close(res9[6], ref['dcpa'], RPZ)
    assert ok, msg


@pytest.mark.parametrize('n', [0, 1, 2, 3, 63, 64, 65, 511, 512, 513, 1025])
def test_ragged_sizes(ctx, n):
    t = synth.box(n, 20.0 + n / 10.0, seed=100 + n)
    got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
    if n == 0:   # the reference's np.max over an empty axis raises; the GPU returns empties
        assert all(len(v) == 0 for v in got.values() if v is not None)
        return
    exp = ocd.detect_arrays(t, t, RPZ, HPZ, TLA)
    util.assert_detect_equal(got, exp, RPZ, TLA)


@pytest.mark.parametrize('seed,n,L', [(7, 4000, 500.0), (11, 3000, 120.0), (13, 2500, 40.0)])
def test_random_boxes_vs_oracle(ctx, seed, n, L):
    t = synth.box(n, L, seed=seed)
    got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
    exp = ocd.detect_arrays(t, t, RPZ, HPZ, TLA)
    util.assert_detect_equal(got, exp, RPZ, TLA)


def test_global_vs_oracle(ctx):
    t = synth.global_traffic(4000, seed=3)
    got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
    exp = ocd.detect_arrays(t, t, RPZ, HPZ, TLA)
    util.assert_detect_equal(got, exp, RPZ, TLA)


def test_row_range_is_a_slice(ctx):
    t = synth.box(3000, 150.0, seed=5)
    full = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
    parts = [statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx, row_begin=a, row_end=b)
             for a, b in ((0, 1000), (1000, 1001), (1001, 3000))]
    for k in ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'li', 'lj', 'inconf', 'tcpamax'):
        assert np.array_equal(np.concatenate([p[k] for p in parts]), full[k]), k


def test_other_lookahead_and_zones(ctx):
    t = synth.box(2000, 100.0, seed=17)
    for rpz, hpz, tla in ((3 * 1852.0, 600.0, 120.0), (8 * 1852.0, 1000 * 0.3048, 600.0),
                          (5 * 1852.0, 304.8, 0.0), (5 * 1852.0, 304.8, -10.0)):
        got = statebased.detect_indices(t, t, rpz, hpz, tla, ctx=ctx)
        exp = ocd.detect_arrays(t, t, rpz, hpz, tla)
        util.assert_detect_equal(got, exp, rpz, max(tla, 1.0))


@pytest.mark.slow
def test_full_size_100k_row_sample(ctx):
    """BASELINE size (100k, density-matched box): every GPU pair of 48 sampled
    rows equals the oracle over all 100k columns; the output is sorted and
    consistent with inconf."""
    t = synth.workload('box100k')
    got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
    key = got['ci'].astype(np.int64) * t.ntraf + got['cj']
    assert np.all(np.diff(key) > 0)
    lkey = got['li'].astype(np.int64) * t.ntraf + got['lj']
    assert np.all(np.diff(lkey) > 0)
    assert np.array_equal(np.unique(got['ci']), np.flatnonzero(got['inconf']))
    rows = np.random.default_rng(1).choice(t.ntraf, 48, replace=False)
    rows.sort()
    exp = ocd.detect_arrays(t, t, RPZ, HPZ, TLA, rows=rows, budget_bytes=512 << 20)
    sel = np.isin(got['ci'], rows)
    lsel = np.isin(got['li'], rows)
    sub = dict(ci=got['ci'][sel], cj=got['cj'][sel], li=got['li'][lsel], lj=got['lj'][lsel],
               qdr=got['qdr'][sel], dist=got['dist'][sel], tcpa=got['tcpa'][sel],
               tinconf=got['tinconf'][sel], inconf=got['inconf'][rows], tcpamax=got['tcpamax'][rows])
    util.assert_detect_equal(sub, exp, RPZ, TLA)
    # density-matched box: ~1.4 conflict pairs per aircraft
    assert 0.5 * t.ntraf < len(got['ci']) < 3.0 * t.ntraf


def test_detect_overflow_retry_is_exact(ctx):
    """A tiny candidate list overflows, the detect grows it and retries: the
    result equals the normal run's exactly."""
    t = synth.box(3000, 120.0, seed=43)
    exp = statebased.detect_indices(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, ctx=ctx)
    ctx.set_candidate_capacity(8)
    got = statebased.detect_indices(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, ctx=ctx)
    for k in ('ci', 'cj', 'li', 'lj', 'qdr', 'dist', 'tcpa', 'tinconf', 'inconf', 'tcpamax'):
        assert np.array_equal(np.asarray(got[k]), np.asarray(exp[k])), k


@pytest.mark.parametrize('path', KWIK, ids=[util.case_name(p) for p in KWIK])
def test_kwik_matches_reference_golden(ctx, path):
    """Opt-in flat-earth variant against the reference's detect with
    kwikqdrdist_matrix swapped in; pruned run == unpruned run."""
    own, intr, z = util.load_cd(path)
    rpz, hpz, tla = float(z['rpz']), float(z['hpz']), float(z['tla'])
    got = statebased.detect_indices(own, intr, rpz, hpz, tla, ctx=ctx, kwik=True)
    util.assert_detect_equal(got, z, rpz, tla)
    full = statebased.detect_indices(own, intr, rpz, hpz, tla, ctx=ctx, kwik=True, noprune=True)
    for k in got:
        if got[k] is not None:
            assert np.array_equal(got[k], full[k]), k


def test_kwik_random_box_vs_oracle(ctx):
    t = synth.box(4000, 300.0, seed=47, lat0=60.0, lon0=20.0)
    got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx, kwik=True)
    exp = ocd.detect_arrays(t, t, RPZ, HPZ, TLA, kwik=True)
    util.assert_detect_equal(got, exp, RPZ, TLA)


def test_row_bucket_widths_are_identical(ctx):
    """K2 row buckets (bsa_set_row_bucket): width 1 and 2 overflow on dense rows
    and retry wider, 0 scatters into row segments -- every width gives the
    default width's results bitwise, on a dense cluster and on a golden case
    with stacked identical aircraft."""
    t = synth.box(2500, 40.0, seed=47)        # ~30 conflicts per aircraft
    cases = [(t, t, RPZ, HPZ, TLA)]
    own, intr, z = util.load_cd(util.golden('cd_edge*.npz')[0])
    cases.append((own, intr, float(z['rpz']), float(z['hpz']), float(z['tla'])))
    try:
        for own, intr, rpz, hpz, tla in cases:
            ctx.set_row_bucket(8)
            exp = statebased.detect_indices(own, intr, rpz, hpz, tla, ctx=ctx, with_dcpa=True)
            for w in (0, 1, 2, 64):
                ctx.set_row_bucket(w)
                got = statebased.detect_indices(own, intr, rpz, hpz, tla, ctx=ctx, with_dcpa=True)
                for k in exp:
                    if exp[k] is not None:
                        assert np.array_equal(np.asarray(got[k]), np.asarray(exp[k])), (w, k)
        assert len(exp['ci']) > 0
    finally:
        ctx.set_row_bucket(8)


def _fusion_ctx():
    from bluesky_amd import _lib
    return _lib.Context(0)


@pytest.mark.parametrize('case', ['box4000', 'global4000', 'dense2000'])
def test_fused_exact_equals_own_launch(case):
    """K1b fused into the prefilter's launch (bsa_set_exact_fusion, default on)
    and K1b as its own launch give bitwise identical results; the fused run
    really fused (bsa_exact_fusion_stats), and against the oracle too."""
    t = {'box4000': lambda: synth.box(4000, 150.0, seed=11),
         'global4000': lambda: synth.global_traffic(4000, seed=13),
         'dense2000': lambda: synth.box(2000, 60.0, seed=17)}[case]()
    c = _fusion_ctx()
    try:
        a = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=c)
        st = c.exact_fusion_stats()
        assert st['last'] and st['fused'] >= 1
        c.set_exact_fusion(False)
        b = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=c)
        assert not c.exact_fusion_stats()['last']
    finally:
        c.close()
    for k in a:
        if a[k] is not None:
            assert np.array_equal(a[k], b[k]), k
    util.assert_detect_equal(a, ocd.detect_arrays(t, t, RPZ, HPZ, TLA), RPZ, TLA)


def test_fused_exact_out_of_records_retries_unfused():
    """A wave that flushes more blocks mid-sweep than it can record makes the
    detect retry with K1b's own launch (max_records 0: any mid-sweep flush):
    the results are those of the fused run, and the next detect fuses again."""
    t = synth.box(3000, 100.0, seed=19)   # dense (<= 29 conflicts a row): waves flush full stages mid-sweep
    c = _fusion_ctx()
    try:
        a = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=c)
        c.set_exact_fusion(True, 0)
        b = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=c)
        st = c.exact_fusion_stats()
        assert st['retries'] >= 1 and not st['last']
        c.set_exact_fusion(True, 64)
        d = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=c)
        assert c.exact_fusion_stats()['last']
    finally:
        c.close()
    for k in a:
        if a[k] is not None:
            assert np.array_equal(a[k], b[k]), k
            assert np.array_equal(a[k], d[k]), k


@pytest.mark.parametrize('field,value', [('lat', np.nan), ('lon', np.nan), ('gs', np.nan), ('trk', np.nan),
                                         ('alt', np.nan), ('vs', np.nan), ('gs', np.inf), ('alt', np.inf)])
def test_nonfinite_aircraft(ctx, field, value):
    """One aircraft with a non-finite state value (a null / erased field): the
    reference's pairs are the finite aircraft's (every comparison with NaN is
    false), and tcpamax = np.max(tcpa * swconfl, axis=1) (StateBasedCD.py:90)
    is NaN on EVERY row once one tcpa is NaN -- an aircraft with a non-finite
    lat / lon / gs / trk makes its whole column NaN."""
    t = synth.box(600, 40.0, seed=23)
    getattr(t, field)[7] = value
    exp = ocd.detect_arrays(t, t, RPZ, HPZ, TLA)
    try:
        for width in (8, 0):   # row buckets (K2 = k_rank_rows) and the scatter path (k_rank)
            ctx.set_row_bucket(width)
            got = statebased.detect_indices(t, t, RPZ, HPZ, TLA, ctx=ctx)
            util.assert_detect_equal(got, exp, RPZ, TLA)
    finally:
        ctx.set_row_bucket(8)


def test_nonfinite_intruder_and_ownship_sets(ctx):
    """Distinct ownship / intruder sets (equal sizes: the reference's
    column-indexed lat == 0 term broadcasts ownship against intruder,
    geo.py:128): the column of aircraft j reads intruder lat / lon and
    ownship gs / trk, its row ownship lat / lon and intruder gs / trk -- a NaN
    in a column input poisons every row's tcpamax, one in a row input only
    that row's."""
    own = synth.box(400, 40.0, seed=29)
    intr = synth.box(400, 40.0, seed=31)
    for who, arr, k in ((own, 'lat', 4), (own, 'gs', 6), (intr, 'lat', 8), (intr, 'trk', 9)):
        t2 = synth.Traffic(*(getattr(who, f).copy() for f in ('lat', 'lon', 'alt', 'trk', 'gs', 'vs')))
        getattr(t2, arr)[k] = np.nan
        o, i = (t2, intr) if who is own else (own, t2)
        exp = ocd.detect_arrays(o, i, RPZ, HPZ, TLA)
        try:
            for width in (8, 0):
                ctx.set_row_bucket(width)
                got = statebased.detect_indices(o, i, RPZ, HPZ, TLA, ctx=ctx)
                util.assert_detect_equal(got, exp, RPZ, TLA)
        finally:
            ctx.set_row_bucket(8)
