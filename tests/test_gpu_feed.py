"""GPU: the resident sim's ACDATA feed (bsa_sim_acdata_*)
against the state it snapshots and the oracle.

ScreenIO.send_aircraft_data (bluesky/simulation/qtgl/screenio.py:194-239)
streams lat lon alt tas cas gs trk vs, asas.inconf / tcpamax, the four pair
counts and asasn / asase.  The feed must equal, bit for bit, what bsa_sim_read
/ bsa_sim_asas_stats return at the same point of the step sequence; inconf /
tcpamax must be the last CD call's (checked against the oracle detect of the
pre-step state); cas = vtas2cas(tas after the step, alt before it)
(traffic.py:434, before UpdatePosition moves alt).
"""
import numpy as np
import pytest

from bluesky_amd import _lib, resident, synth
from oracle import kinematics as okin
from oracle import statebased as ocd
from tests import util

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('resume_nav', [False, True])
def test_acdata_matches_state_and_oracle(ctx, resume_nav):
    t = synth.box(2000, 80.0, seed=61)
    init = resident.initial_state(t)
    sim = resident.ResidentSim(init, resident.params(resume_nav=resume_nav), ctx=ctx)
    sim.step(3)
    pre = sim.read()
    sim.step(1)
    sim.acdata_request()
    got = sim.acdata(wait=True)
    post = sim.read()
    assert got['steps'] == 4 and (got['row_begin'], got['row_end']) == (0, t.ntraf)
    for k in ('lat', 'lon', 'alt', 'tas', 'gs', 'trk', 'vs'):
        assert np.array_equal(got[k], post[k]), k
    # cas after the step: vtas2cas(new tas, old alt)
    ok, msg = util.close(got['cas'], okin.vtas2cas(post['tas'], pre['alt']), 300.0)
    assert ok, msg
    # inconf / tcpamax of the CD call at the start of step 4 (on the pre-step state)
    s = synth.Traffic(pre['lat'], pre['lon'], pre['alt'], pre['trk'], pre['gs'], pre['vs'])
    exp = ocd.detect_arrays(s, s, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD)
    assert np.array_equal(got['inconf'], exp['inconf'])
    assert util.close(got['tcpamax'], exp['tcpamax'], synth.TLOOKAHEAD)[0]
    assert got['inconf'].any()
    assert np.any(got['asase'] != 0) and got['asasn'].dtype == np.float32
    if resume_nav:
        st = sim.asas_stats()
        assert (got['nconf_cur'], got['nlos_cur'], got['nconf_tot'], got['nlos_tot']) == \
            (st['confpairs_unique'], st['lospairs_unique'], st['confpairs_all'], st['lospairs_all'])
    else:
        assert got['nconf_cur'] == got['nconf_tot'] == got['nlos_cur'] == got['nlos_tot'] == -1


def test_acdata_poll_without_wait_and_ordering(ctx):
    """A snapshot requested behind queued steps reflects exactly those steps;
    polling without waiting returns None or the finished snapshot."""
    t = synth.box(3000, 120.0, seed=62)
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(), ctx=ctx)
    sim.step(2)
    sim.acdata_request()
    sim.step(5)                    # queued behind the snapshot
    got = None
    for _ in range(200000):
        got = sim.acdata(wait=False)
        if got is not None:
            break
    assert got is not None and got['steps'] == 2
    ctx.sync()
    sim.acdata_request()
    now = sim.acdata(wait=True)
    assert now['steps'] == 7
    assert np.array_equal(now['lat'], sim.read()['lat'])
    assert not np.array_equal(now['lat'], got['lat'])


def test_acdata_before_any_step_and_errors(ctx):
    t = synth.box(100, 20.0, seed=63)
    init = resident.initial_state(t)
    sim = resident.ResidentSim(init, resident.params(), ctx=ctx)
    with pytest.raises(_lib.AccelError, match='no ACDATA snapshot'):
        sim.acdata()
    sim.acdata_request()
    got = sim.acdata()
    assert got['steps'] == 0
    assert np.array_equal(got['lat'], init['lat'])
    assert not got['inconf'].any() and np.all(got['tcpamax'] == 0.0) and np.all(got['cas'] == 0.0)
