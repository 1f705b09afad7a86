"""CPU: the lake module of the RHS in the oracle, on qhh (688 lake elements, one lake,
bank edges) and a qhh variant with reaches redirected into the lake.

Checks the restatement against the reference's own bookkeeping identities, recomputed here in plain Python
in the reference's loop order (bit for bit): lake-element DY is zero (MD_f.cpp:146-150); QLakeSurf/QLakeSub
are the bank edges' fluxes summed in element-then-edge order (MD_ElementFlux.cpp:52,121); QLakeRivIn sums
QrivDown of the inflowing reaches (MD_RiverFlux.cpp:24); qLakeEvap/qLakePrcp are the lake elements' means
with the evaporation clamp (MD_f.cpp:16-17,44-47); the lake DY is MD_f.cpp:180-183; lake elements carry
qEleE_IC = 0 and u_satn = 1 (fun_Ele_lakeVertical, updateLakeElement).  OMP + lakes is rejected."""
import numpy as np
import pytest

import cases
import oracle
from shud_rhs import abi


def _bank_edges(m):
    NE = m.num_ele
    nab = m.nabr.reshape(3, NE)
    out = []
    for i in range(NE):
        if m.ilake[i] > 0:
            continue
        for j in range(3):
            nb = nab[j, i]
            if nb >= 0 and m.ilake[nb] > 0:
                out.append((i, j, m.ilake[nb] - 1))
    return out


@pytest.mark.parametrize("case", ["qhh", "qhh_variant"])
def test_lake_bookkeeping(case):
    m, y = getattr(cases, case)()
    NE, NR, NL = m.num_ele, m.num_riv, m.num_lake
    assert NL == 1 and (m.ilake > 0).sum() == 688
    o = oracle.OracleRhs(m, abi.SHUD_MODE_SERIAL)
    o.set_step_inputs()
    ys = [y.copy(), y.copy()]
    ys[1][-1] = 300.0                                          # lake level above the bank: weir exchange
    for yy in ys:
        for call in range(2):
            dy, code, _, _ = o.eval(0.0, yy)
            assert code == 0
            d = o.diagnostics()
            lake = m.ilake > 0
            assert np.all(dy[:NE][lake] == 0) and np.all(dy[NE:2 * NE][lake] == 0) and np.all(dy[2 * NE:3 * NE][lake] == 0)
            assert np.all(d["e_ic"][lake] == 0) and np.all(d["u_satn"][lake] == 1)
            qs = qg = 0.0
            qsurf, qsub = d["qele_surf"].reshape(3, NE), d["qele_sub"].reshape(3, NE)
            fu = m.step["fu_sub"]
            for i, j, l in _bank_edges(m):
                qs += qsurf[j, i]
                if np.all(fu == 1.0):
                    qg += qsub[j, i]
            assert d["q_lake_surf"][0] == qs
            if np.all(fu == 1.0):
                assert d["q_lake_sub"][0] == qg
            rin = 0.0
            for r in range(NR):
                if m.riv_down[r] <= -4:
                    rin += d["qriv_down"][r]
            assert d["q_lake_rivin"][0] == rin
            n = float(lake.sum())
            qe = qp = 0.0
            for i in np.nonzero(lake)[0]:
                qe += m.step["pot_evap"][i] / n
                qp += m.step["prcp"][i] / n
            stage = yy[3 * NE + NR]
            qe = (qp + stage) if qe > qp + stage else qe       # min(a, b) = a > b ? b : a
            qe = qe if 0 < qe else 0.0                           # max(0, a) = 0 < a ? a : 0
            assert d["q_lake_evap"][0] == qe and d["q_lake_prcp"][0] == qp
            want = qp - qe + (rin - 0. + d["q_lake_sub"][0] + d["q_lake_surf"][0]) / d["lake_toparea"][0]
            assert dy[3 * NE + NR] == want
    assert len(_bank_edges(m)) > 0


def test_lake_toparea_interpolation():
    """LakeBathymetry::toparea (Lake.cpp:59-79) on qhh's table, below / inside / above the rows."""
    m, y = cases.qhh()
    o = oracle.OracleRhs(m, abi.SHUD_MODE_SERIAL)
    o.set_step_inputs()
    yi, ai = m.lake_bathy_y, m.lake_bathy_a
    for stage in [-5.0, 0.0, 5.0, 10.0, 45.0, 79.9, 80.0, 200.0]:
        yy = y.copy()
        yy[-1] = stage
        o.eval(0.0, yy)
        got = o.diagnostics()["lake_toparea"][0]
        yv = stage + yi[0]
        ta = ai[0]
        if not yv <= yi[0]:
            for k in range(1, yi.size):
                if yv < yi[k]:
                    ta = (ai[k] - ta) / (yi[k] - yv) * (yv - yi[k - 1]) + ta
                    break
                ta = ai[k]
        assert got == ta, stage


def test_lake_omp_rejected():
    m, _ = cases.qhh()
    with pytest.raises(ValueError):
        oracle.OracleRhs(m, abi.SHUD_MODE_OMP)
