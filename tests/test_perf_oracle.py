"""CPU: OpenAP flight phase / envelope / acceleration (perfoap.py:115-131,
211-280; phase.py:14-62) -- the oracle and the host-side type table against
tests/golden/perf_openap3000.npz, captured from the reference's own functions
on its own coefficient tables (tools/make_golden.py run_perf)."""
import numpy as np

from bluesky_amd import perf
from oracle import perf as operf
from tests import util

FIXWING_FIELDS = ('vminto', 'vmaxto', 'vminic', 'vmaxic', 'vminer', 'vmaxer', 'vminap', 'vmaxap', 'vminld',
                  'vmaxld', 'vsmin', 'vsmax', 'hmax', 'axmax')
ROTOR_FIELDS = ('vmin', 'vmax', 'vsmin', 'vsmax', 'hmax')


def load():
    g = dict(np.load(util.golden('perf_openap3000.npz')[0]))
    fw = {str(m): {f: float(g['fw_' + f][k]) for f in FIXWING_FIELDS} for k, m in enumerate(g['fw_types'])}
    rot = {str(m): {f: float(g['rot_' + f][k]) for f in ROTOR_FIELDS} for k, m in enumerate(g['rot_types'])}
    return g, fw, rot


def test_oracle_phase_limits_accel_match_reference():
    g, fw, rot = load()
    ph = operf.phase(g['lifttype'], g['tas'], g['vs'], g['alt'])
    assert np.array_equal(ph, g['phase'])
    lim = operf.limit_matrix(fw, rot, g['actypes'], g['lifttype'], ph)
    assert np.array_equal(lim, g['limits'])
    assert np.array_equal(operf.acceleration(ph), g['accel'])
    # the fixture reaches every phase the reference can produce (TO / LD never are: phase.py:56-61)
    assert set(np.unique(g['phase']).astype(int)) == {perf.NA, perf.IC, perf.CL, perf.CR, perf.DE, perf.AP, perf.GD}
    assert (g['lifttype'] == perf.LIFT_ROTOR).any()


def test_type_table_lookup_matches_reference():
    """The table bsa_sim_set_perf uploads, looked up the way K4' does
    (row tidx, column phase / 9 + phase / 18..21), gives the reference's matrix."""
    g, fw, rot = load()
    table, tidx = perf.type_table(fw, rot, g['actypes'], g['lifttype'])
    assert table.shape == (len(fw) + len(rot), perf.PERF_COLS) and tidx.dtype == np.int32
    ph = g['phase'].astype(int)
    row = table[tidx]
    n = np.arange(len(ph))
    got = np.stack([row[n, ph], row[n, 9 + ph], row[:, 18], row[:, 19], row[:, 20], row[:, 21]], axis=1)
    assert np.array_equal(got, g['limits'])
    assert np.array_equal(row[:, 22], g['lifttype'].astype(float))


def test_type_table_other_lift_type_is_zero():
    table, tidx = perf.type_table({}, {}, ['XXXX', 'XXXX'], [0, 0])
    assert table.shape == (1, perf.PERF_COLS) and not table.any() and tidx.tolist() == [0, 0]
