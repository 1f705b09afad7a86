"""GPU: the ET-step prelude on the device (shud_et_step, include/shud_et.h).

(1) Device prelude vs the CPU restatement (oracle/shud_oracle_et.c) over multi-step sequences: every output
    within the parity tolerance (OCML vs glibc exp/log ulps), all configurations (cryosphere queues, SWNET,
    terrain-radiation modes, lakes, LAI = 0).
(2) The prelude writes the RHS step inputs in place: RHS evaluations after shud_et_step equal the oracle RHS
    fed with the prelude's own outputs (both layouts), across ET steps and stateful RHS calls.
(3) The reference's exits from tReadForcing (CheckNonZero(ra), CheckNANi(qPotTran)) -> code 10, first element."""
import numpy as np
import pytest

import cases
import oracle
from conftest import assert_close, rhs_blocks
from shud_rhs import abi, et, workload

pytestmark = pytest.mark.gpu

KEYS = ["t_prcp", "t_temp", "t_lai", "t_mf", "t_rn", "t_wind", "t_rh", "qEleprep", "qPotEvap", "qPotTran",
        "qEleETP", "qEleNetPrep", "qEleE_IC", "yEleIS", "yEleSnow", "fu_surf", "fu_sub", "rn_factor"]


def _seq(n):
    out = []
    for k in range(n):
        mode = abi.SHUD_TSR_RECOMPUTE if k % 4 == 0 else abi.SHUD_TSR_CACHED
        if k == 6:
            mode = abi.SHUD_TSR_NO_TIME
        out.append((360.0 * k, mode))
    return out


@pytest.fixture(params=["packed", "soa"])
def layout(request, monkeypatch):
    monkeypatch.setenv("SHUD_RHS_PACKED", "1" if request.param == "packed" else "0")
    return request.param


@pytest.mark.parametrize("cryo,swnet,terrain", [(0, 0, 1), (1, 0, 1), (1, 1, 0)])
def test_device_et_vs_oracle_and_rhs_chain(cryo, swnet, terrain, layout):
    from shud_rhs import runtime as rt
    m, y = cases.variant(20000, seed=17)
    etm = et.synth_et(m.num_ele, seed=4, terrain=bool(terrain), lake_frac=0.03)
    etm.params.update(cryosphere=cryo, radiation_input_mode=swnet, ft_surf_day=3, ft_sub_day=5)
    h = rt.RhsHandle(m, mode=abi.SHUD_MODE_SERIAL)
    assert h.layout()["packed"] == (layout == "packed")
    h.set_step_inputs()
    h.et_attach(etm)
    oe = oracle.OracleEt(etm)
    orc = oracle.OracleRhs(m, abi.SHUD_MODE_SERIAL)
    orc.set_step_inputs()
    rng = np.random.default_rng(2)
    y_is = rng.uniform(0, 2e-4, m.num_ele)
    y_snow = np.where(rng.random(m.num_ele) < 0.5, 0.0, rng.uniform(0, 0.05, m.num_ele))
    h.et_set_state(y_is, y_snow)
    oe.set_state(y_is, y_snow)
    ys = [y, workload.random_state(m, seed=5)]
    for k, (t, mode) in enumerate(_seq(9)):
        f = et.synth_forcing(t, 360.0, seed=k, tsr_mode=mode if terrain else abi.SHUD_TSR_OFF)
        assert h.et_step(f) == abi.SHUD_OK
        assert oe.step(f) == (0, -1)
        got, ref = h.et_get(), oe.get()
        for key in KEYS:
            assert_close(got[key], ref[key], what=f"step {k} {key}")
        # the RHS now runs on the device-written step inputs; the oracle RHS gets the same values
        orc.set_step_inputs(step=dict(net_prep=got["qEleNetPrep"], pot_evap=got["qPotEvap"],
                                      pot_tran=got["qPotTran"], etp=got["qEleETP"], lai=got["t_lai"],
                                      fu_surf=got["fu_surf"], fu_sub=got["fu_sub"], e_ic=got["qEleE_IC"]))
        for c in range(2):
            yy = ys[(k + c) % 2]
            ref_dy, code, _, _ = orc.eval(t, yy)
            assert code == 0
            assert_close(h.eval(t, yy), ref_dy, what=f"rhs after ET step {k} call {c}", blocks=rhs_blocks(m))
    h.close()


@pytest.mark.parametrize("what,bit,slot", [("wind_nan", abi.EF_ET_RA, 5), ("temp_nan", abi.EF_ET_PT_NAN, 6)])
def test_device_et_exits(what, bit, slot):
    from shud_rhs import runtime as rt
    m, _ = cases.variant(5000, seed=3)
    etm = et.synth_et(m.num_ele, seed=9, terrain=False)
    h = rt.RhsHandle(m)
    h.set_step_inputs()
    h.et_attach(etm)
    f = et.synth_forcing(0.0, 60.0, seed=2)
    st = f.station.copy()
    st[:, 4 if what == "wind_nan" else 2] = np.nan
    f.station = st
    code, idx = oracle.OracleEt(etm).step(f)
    assert code == 10
    with pytest.raises(rt.ShudRhsError) as ei:
        h.et_step(f)
    e = ei.value.err
    assert e["exit_code"] == 10 and e["flags"] & bit and e["first_index"][slot] == idx, e
    h.close()
