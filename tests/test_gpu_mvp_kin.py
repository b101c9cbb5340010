"""GPU parity: bsa_mvp (K3) and bsa_kinematics (K4) against the reference's
golden vectors (tests/golden/mvp_*.npz, kin_*.npz), 1e-9 relative."""
import numpy as np
import pytest

from bluesky_amd import _lib
from tests import util
from tests.test_oracle_golden import MODE_SW, MODES

pytestmark = pytest.mark.gpu

MVP = util.golden('mvp_*.npz')
KIN = util.golden('kin_*.npz')

FT = 0.3048
NM = 1852.0


def mvp_params(z, mode):
    hz, spd, hdg, vert, prio, code = MODE_SW[mode]
    mar = float(z['mar'])
    R, dh = float(z['rpz']), float(z['hpz'])
    return _lib.MvpParams(Rm=R * mar, dhm=dh * mar, dtlookahead=float(z['tla']),
                          vmin=200.0 * NM / 3600., vmax=500.0 * NM / 3600.,
                          vsmin=-3000. / 60. * FT, vsmax=3000. / 60. * FT,
                          swresohoriz=int(hz), swresospd=int(spd), swresohdg=int(hdg),
                          swresovert=int(vert), swprio=int(prio),
                          priocode=_lib.PRIO_CODES.get(code, 0),
                          swnoreso=int(mode == 'noreso'), swresooff=int(mode == 'resooff'))


@pytest.mark.parametrize('path', MVP, ids=[util.case_name(p) for p in MVP])
def test_mvp_matches_reference_golden(ctx, path):
    z = dict(np.load(path, allow_pickle=False))
    n = len(z['alt'])
    ctx.set_state(z['lat'], z['lon'], z['trk'], z['gs'], z['alt'], z['vs'])
    ctx.set_pairs(z['ci'], z['cj'], z['qdr'], z['dist'], z['tcpa'], z['tLOS'])
    noreso_mask = np.isin(np.arange(n), z['noreso_idx'])
    resooff_mask = np.isin(np.arange(n), z['resooff_idx'])
    for mode in MODES:
        alt = np.ascontiguousarray(z['asasalt'], dtype=np.float64).copy()
        o = ctx.mvp(mvp_params(z, mode), z['gseast'], z['gsnorth'], z['selalt'], z['apvs'], alt,
                    noreso=noreso_mask, resooff=resooff_mask)
        o['alt'] = alt
        for k, scale in (('trk', 360.0), ('tas', 300.0), ('vs', 20.0), ('alt', 1e4),
                         ('asase', 300.0), ('asasn', 300.0)):
            exp = z['%s__%s' % (mode, k)]
            if k in ('asase', 'asasn'):
                # float32 outputs: one float32 rounding of an fp64 value that
                # agrees to 1e-9 -> equal or 1 float32 ulp apart
                ok, msg = util.close(o[k], exp, scale, rtol=2 ** -23)
            else:
                ok, msg = util.close(o[k], exp, scale)
            assert ok, '%s/%s: %s' % (mode, k, msg)


def test_mvp_after_gpu_detect(ctx):
    """MVP consuming the device-resident pairs of bsa_detect directly."""
    path = util.golden('mvp_box500.npz')[0]
    z = dict(np.load(path, allow_pickle=False))
    ctx.set_state(z['lat'], z['lon'], z['trk'], z['gs'], z['alt'], z['vs'])
    nc, nl = ctx.detect(float(z['rpz']), float(z['hpz']), float(z['tla']))
    assert nc == len(z['ci'])
    alt = np.ascontiguousarray(z['asasalt'], dtype=np.float64).copy()
    o = ctx.mvp(mvp_params(z, 'default'), z['gseast'], z['gsnorth'], z['selalt'], z['apvs'], alt)
    ok, msg = util.close(o['trk'], z['default__trk'], 360.0)
    assert ok, msg
    ok, msg = util.close(alt, z['default__alt'], 1e4)
    assert ok, msg


@pytest.mark.parametrize('path', KIN, ids=[util.case_name(p) for p in KIN])
def test_kinematics_matches_reference_golden(ctx, path):
    z = dict(np.load(path, allow_pickle=False))
    state = {k: np.ascontiguousarray(z[k], dtype=np.float64).copy()
             for k in ('tas', 'hdg', 'alt', 'vs', 'lat', 'lon')}
    inputs = {k: z[k] for k in ('ptas', 'phdg', 'palt', 'pvs', 'bank', 'eps', 'accel')}
    wd = int(z['winddim'])
    if wd == 2:   # 2-D wind field (bsa_set_windfield), the reference's getdata pinned by the fixture
        ctx.set_windfield(z['wlat'], z['wlon'], z['wvnorth'], z['wveast'])
        o = ctx.kinematics(float(z['dt']), state, inputs, 2, 0.0, 0.0)
        ctx.set_windfield()
    else:
        o = ctx.kinematics(float(z['dt']), state, inputs, wd, float(z['windnorth']), float(z['windeast']))
    o.update(state)
    o['M'] = o.pop('mach')
    scales = dict(ax=1.0, delspd=100.0, tas=300.0, cas=300.0, M=1.0, hdg=360.0, az=1.0, vs=20.0,
                  gsnorth=300.0, gseast=300.0, gs=300.0, trk=360.0, alt=1e4, lat=90.0, lon=180.0,
                  coslat=1.0)
    for k, s in scales.items():
        ok, msg = util.close(o[k], z['out_' + k], s)
        assert ok, '%s: %s' % (k, msg)
    for k in ('swhdgsel', 'swaltsel'):
        assert np.array_equal(o[k], z['out_' + k].astype(bool)), k


@pytest.mark.parametrize('path', MVP, ids=[util.case_name(p) for p in MVP])
def test_mvp_dropin_resolve_matches_reference_golden(ctx, path):
    """The CR drop-in a BlueSky user registers (bluesky_amd.mvp.resolve(asas, traf),
    MVP.py:14-143) on SimpleNamespace stand-ins: confpairs as id tuples (here in a
    shuffled order that keeps each ownship's pairs in their original relative
    order, as any CD's row-major output does), NORESO / RESOOFF as id lists."""
    import types
    from bluesky_amd import mvp
    z = dict(np.load(path, allow_pickle=False))
    n = len(z['alt'])
    ids = ['KL%04d' % k for k in range(n)]
    P = len(z['ci'])
    order = np.argsort(np.random.default_rng(3).permutation(n)[z['ci']], kind='stable')
    traf = types.SimpleNamespace(ntraf=n, id=ids, lat=z['lat'], lon=z['lon'], trk=z['trk'], gs=z['gs'],
                                 alt=z['alt'], vs=z['vs'], gseast=z['gseast'], gsnorth=z['gsnorth'],
                                 selalt=z['selalt'], ap=types.SimpleNamespace(vs=z['apvs']))
    for mode in MODES:
        hz, spd, hdg, vert, prio, code = MODE_SW[mode]
        asas = types.SimpleNamespace(
            swasas=True, asaseval=False, Rm=float(z['rpz']) * float(z['mar']),
            dhm=float(z['hpz']) * float(z['mar']), dtlookahead=float(z['tla']),
            vmin=200.0 * NM / 3600., vmax=500.0 * NM / 3600., vsmin=-3000. / 60. * FT, vsmax=3000. / 60. * FT,
            swresohoriz=hz, swresospd=spd, swresohdg=hdg, swresovert=vert, swprio=prio, priocode=code,
            swnoreso=mode == 'noreso', noresolst=[ids[k] for k in z['noreso_idx']],
            swresooff=mode == 'resooff', resoofflst=[ids[k] for k in z['resooff_idx']],
            confpairs=[(ids[z['ci'][k]], ids[z['cj'][k]]) for k in order], qdr=z['qdr'][order],
            dist=z['dist'][order], tcpa=z['tcpa'][order], tLOS=z['tLOS'][order], alt=z['asasalt'].copy())
        mvp.resolve(asas, traf, ctx=ctx)
        assert asas.asaseval or P == 0
        for k, scale in (('trk', 360.0), ('tas', 300.0), ('vs', 20.0), ('alt', 1e4)):
            ok, msg = util.close(getattr(asas, k), z['%s__%s' % (mode, k)], scale)
            assert ok, '%s/%s: %s' % (mode, k, msg)
        for k in ('asase', 'asasn'):
            ok, msg = util.close(getattr(asas, k), z['%s__%s' % (mode, k)], 300.0, rtol=2 ** -23)
            assert ok, '%s/%s: %s' % (mode, k, msg)


@pytest.mark.parametrize('path', KIN, ids=[util.case_name(p) for p in KIN])
def test_kinematics_dropin_install_matches_reference_golden(ctx, path):
    """kinematics.install(traf) rebinds Traffic.UpdateAirSpeed / UpdateGroundSpeed /
    UpdatePosition (traffic.py:425-483) on the instance; Traffic.update's three
    calls (traffic.py:407-409) then produce the reference's arrays."""
    import types
    from bluesky_amd import kinematics
    z = dict(np.load(path, allow_pickle=False))
    wd = int(z['winddim'])
    wind = types.SimpleNamespace(winddim=wd)
    if wd == 1:
        wind.vnorth = np.array([[float(z['windnorth'])]])
        wind.veast = np.array([[float(z['windeast'])]])
    elif wd == 2:
        wind.lat, wind.lon = z['wlat'], z['wlon']
        wind.vnorth, wind.veast = z['wvnorth'][None, :], z['wveast'][None, :]
    acc = z['accel'].copy()
    traf = types.SimpleNamespace(
        pilot=types.SimpleNamespace(tas=z['ptas'], hdg=z['phdg'], alt=z['palt'], vs=z['pvs']),
        perf=types.SimpleNamespace(acceleration=lambda: acc), wind=wind, bank=z['bank'], eps=z['eps'],
        tas=z['tas'].copy(), hdg=z['hdg'].copy(), alt=z['alt'].copy(), vs=z['vs'].copy(),
        lat=z['lat'].copy(), lon=z['lon'].copy())
    kinematics.install(traf, ctx=ctx)
    dt = float(z['dt'])
    traf.UpdateAirSpeed(dt, 0.0)
    traf.UpdateGroundSpeed(dt)
    traf.UpdatePosition(dt)
    if wd == 2:
        ctx.set_windfield()
    scales = dict(ax=1.0, delspd=100.0, tas=300.0, cas=300.0, M=1.0, hdg=360.0, az=1.0, vs=20.0,
                  gsnorth=300.0, gseast=300.0, gs=300.0, trk=360.0, alt=1e4, lat=90.0, lon=180.0,
                  coslat=1.0)
    for k, s in scales.items():
        ok, msg = util.close(getattr(traf, k), z['out_' + k], s)
        assert ok, '%s: %s' % (k, msg)
    for k in ('swhdgsel', 'swaltsel'):
        assert np.array_equal(getattr(traf, k), z['out_' + k].astype(bool)), k
