"""ET-step prelude (include/shud_et.h).

CPU: the C restatement (oracle/shud_oracle_et.c) equals the independent pure-Python restatement
(tests/et_py.py) bit for bit over multi-step sequences covering lakes, LAI = 0, NA station elevation,
RH clamps, rain/snow/melt regimes, SWDOWN/SWNET, every TSR mode and the cryosphere day-mean queues; and the
reference's exits (CheckNonZero(ra), CheckNANi(qPotTran) -> 10) at the first element in loop order."""
import numpy as np
import pytest

import oracle
from et_py import PyEt
from shud_rhs import abi, et

KEYS = ["t_prcp", "t_temp", "t_lai", "t_mf", "t_rn", "t_wind", "t_rh", "qEleprep", "qPotEvap", "qPotTran",
        "qEleETP", "qEleNetPrep", "qEleE_IC", "yEleIS", "yEleSnow", "fu_surf", "fu_sub", "rn_factor"]


def _seq(n_steps):
    """(t, tsr_mode) sequence: a new forcing interval every 4 steps, one step without forcing time"""
    out = []
    for k in range(n_steps):
        mode = abi.SHUD_TSR_RECOMPUTE if k % 4 == 0 else abi.SHUD_TSR_CACHED
        if k == 6:
            mode = abi.SHUD_TSR_NO_TIME
        out.append((360.0 * k, mode))
    return out


def _bitwise(a, b):
    return np.array_equal(a, b) or bool(((a == b) | (np.isnan(a) & np.isnan(b))).all())


@pytest.mark.parametrize("cryo,swnet,terrain", [(0, 0, 1), (1, 0, 1), (1, 1, 0)])
def test_oracle_et_vs_python(cryo, swnet, terrain):
    etm = et.synth_et(240, seed=5, terrain=bool(terrain), lake_frac=0.05)
    etm.params.update(cryosphere=cryo, radiation_input_mode=swnet, ft_surf_day=3, ft_sub_day=5)
    o, py = oracle.OracleEt(etm), PyEt(etm)
    rng = np.random.default_rng(1)
    y_is, y_snow = rng.uniform(0, 2e-4, 240), np.where(rng.random(240) < 0.5, 0.0, rng.uniform(0, 0.05, 240))
    o.set_state(y_is, y_snow)
    py.y_is[:], py.y_snow[:] = y_is, y_snow
    for k, (t, mode) in enumerate(_seq(10)):
        f = et.synth_forcing(t, 360.0, seed=k, tsr_mode=mode if terrain else abi.SHUD_TSR_OFF)
        assert o.step(f) == (0, -1)
        assert py.step(f) == (0, -1)
        got = o.get()
        for key in KEYS:
            assert _bitwise(got[key], py.out[key]), f"step {k} {key}"


@pytest.mark.parametrize("what", ["wind_nan", "temp_nan"])
def test_oracle_et_exits(what):
    etm = et.synth_et(200, seed=9, terrain=False)
    f = et.synth_forcing(0.0, 60.0, seed=2)
    st = f.station.copy()
    if what == "wind_nan":        # Uz NaN -> ra NaN -> CheckNonZero -> exit 10
        st[:, 4] = np.nan
    else:                         # TMP NaN -> qPotTran NaN (ra is fine) -> CheckNANi -> exit 10
        st[:, 2] = np.nan
    f.station = st
    lai = etm.arrays["ilc"]
    first_veg = int(np.nonzero((f.lai_row[lai] > 0) & (etm.arrays["ilake"] == 0))[0][0])
    o, py = oracle.OracleEt(etm), PyEt(etm)
    assert o.step(f) == (10, first_veg)
    assert py.step(f) == (10, first_veg)
