"""GPU: the device output path (include/shud_out.h) against the Print_Ctrl restatement
(tests/print_ctrl_py.py) fed with the same values read back from the handle: Model_Data::summary on the
device (MD_update.cpp:190-216, BC overrides), the replayed diagnostics of the last RHS call, and the
ET-step inputs.  The files must be identical byte for byte (binary) and line for line (ASCII): the device
sums and scales in the reference's order."""
import numpy as np
import pytest

import cases
from print_ctrl_py import PrintCtrlPy
from shud_rhs import abi, workload
from shud_rhs import runtime as rt
from shud_rhs.shudio import read_dat

pytestmark = pytest.mark.gpu


def _host_summary(m, y):
    NE, NR = m.num_ele, m.num_riv
    ybc, rbc = m.bc_tables.get("ele_ybc"), m.bc_tables.get("riv_ybc")
    gw = y[2 * NE:3 * NE].copy()
    stg = y[3 * NE:3 * NE + NR].copy()
    ibc = np.asarray(m.ibc)
    if ybc is not None and (ibc > 0).any():
        gw[ibc > 0] = ybc[ibc[ibc > 0]]
    rb = np.asarray(m.riv_bc)
    if rbc is not None and (rb > 0).any():
        stg[rb > 0] = rbc[rb[rb > 0]]
    return {abi.SHUD_ARR_Y_ELE_SURF: y[:NE], abi.SHUD_ARR_Y_ELE_UNSAT: y[NE:2 * NE], abi.SHUD_ARR_Y_ELE_GW: gw,
            abi.SHUD_ARR_Y_RIV_STG: stg}


@pytest.mark.parametrize("case", ["ccw", "variant"])
def test_device_outputs_match_restatement(tmp_path, case):
    m, y0 = cases.ccw() if case == "ccw" else cases.variant()
    if case == "ccw":
        m.step = workload.random_step_inputs(m, seed=3)
    NE, NR = m.num_ele, m.num_riv
    h = rt.RhsHandle(m)
    h.set_step_inputs()
    dy, ddy = h.device_alloc(8 * m.num_y), h.device_alloc(8 * m.num_y)
    out = rt.Output(stream=h.stream())
    rng = np.random.default_rng(5)
    flags = (rng.random(NE) < 0.7).astype(np.int32)
    # (array, column, interval, iflux, flag_io, ascii): element/river storages, fluxes, InitIJ columns, inputs
    specs = [(abi.SHUD_ARR_Y_ELE_SURF, 0, 60, 0, None, False), (abi.SHUD_ARR_Y_ELE_GW, 0, 60, 0, flags, True),
             (abi.SHUD_ARR_Y_RIV_STG, 0, 120, 0, None, False), (abi.SHUD_ARR_QELE_SURF_TOT, 0, 1440, 1, None, True),
             (abi.SHUD_ARR_QELE_SUB, 2, 1440, 1, flags, False), (abi.SHUD_ARR_Q_INFIL, 0, 60, 1, None, False),
             (abi.SHUD_ARR_QRIV_DOWN, 0, 60, 1, None, False), (abi.SHUD_ARR_Q_TRANS, 0, 1440, 1, None, False),
             (abi.SHUD_ARR_Q_EVAPO, 0, 1440, 1, None, False), (abi.SHUD_ARR_Q_PRCP, 0, 1440, 1, None, False)]
    # materialise the device arrays once (summary + diagnostics of a first call)
    h.h2d(dy, y0)
    h.eval_device(0.0, dy, ddy)
    h.summary(dy)
    h.refresh_diagnostics()
    ref = []
    for k, (arr, col, itv, flx, fl, asc) in enumerate(specs):
        p, n = h.device_array(arr)
        assert p, arr
        n_all = NE if arr in (abi.SHUD_ARR_QELE_SURF, abi.SHUD_ARR_QELE_SUB) else n
        base = tmp_path / f"dev{k}"
        out.add(base, p + 8 * col * NE, n_all, itv, flx, start_time=0, flag_io=fl, ascii=asc)
        ref.append((arr, col, PrintCtrlPy(tmp_path / f"ref{k}", n_all, itv, flx, start_time=0, flag_io=fl,
                                          ascii=asc)))
    times = np.concatenate([np.arange(1, 97) * 30.0, [2880.4, 2910.0, 2939.9995]])   # 2 days + off-grid times
    for k, t in enumerate(times):
        y = workload.random_state(m, seed=1000 + k)
        h.h2d(dy, y)
        h.eval_device(t, dy, ddy)
        h.summary(dy)                        # Model_Data::summary(udata)
        h.refresh_diagnostics()              # flux arrays of the last f() call
        out.export(t)                        # ExportResults(t)
        diag = h.diagnostics()
        host = _host_summary(m, y)
        host.update({abi.SHUD_ARR_QELE_SURF_TOT: diag["qele_surf_tot"], abi.SHUD_ARR_QELE_SUB: diag["qele_sub"],
                     abi.SHUD_ARR_Q_INFIL: diag["q_infil"], abi.SHUD_ARR_QRIV_DOWN: diag["qriv_down"],
                     abi.SHUD_ARR_Q_TRANS: diag["q_tg"] + diag["q_tu"],
                     abi.SHUD_ARR_Q_EVAPO: diag["q_eu"] + diag["q_eg"] + diag["q_es"],
                     abi.SHUD_ARR_Q_PRCP: np.asarray(m.step.get("prcp", np.zeros(NE)), dtype=np.float64)})
        for arr, col, p in ref:
            v = host[arr]
            if arr == abi.SHUD_ARR_QELE_SUB:
                v = v[col * NE:(col + 1) * NE]
            p.print_data(v, t)
    rows = [out.rows(k) for k in range(len(specs))]
    out.close()
    for _, _, p in ref:
        p.close()
    assert rows[0] == 50 and rows[2] == 25 and rows[3] == 3, rows
    for k, (arr, col, itv, flx, fl, asc) in enumerate(specs):
        a = open(tmp_path / f"dev{k}.dat", "rb").read()
        b = open(tmp_path / f"ref{k}.dat", "rb").read()
        assert a == b, (k, arr, len(a), len(b), read_dat(tmp_path / f"dev{k}.dat")["data"][:1, :4],
                        read_dat(tmp_path / f"ref{k}.dat")["data"][:1, :4])
        if asc:
            assert open(tmp_path / f"dev{k}.csv").read() == open(tmp_path / f"ref{k}.csv").read(), k
    d = read_dat(tmp_path / "dev3.dat")
    assert d["t"].tolist() == [0.0, 1440.0, 1440.0] and np.isfinite(d["data"]).all()
    h.device_free(dy)
    h.device_free(ddy)
    h.close()


def test_solver_loop_exports_on_device(tmp_path):
    """SHUD()'s loop on the device (ShudSolver): after every solver step summary(udata) on y(tout) and
    ExportResults(t) on the device; the restatement is fed y(tout) and the replayed diagnostics of the
    integrator's last RHS call, read back at the same point."""
    from shud_rhs.solver import ShudSolver, SolverControl
    m, y0 = cases.ccw()
    m.step = workload.random_step_inputs(m, seed=4)
    NE = m.num_ele
    h = rt.RhsHandle(m, mode=abi.SHUD_MODE_OMP)
    h.set_step_inputs()
    out = rt.Output(stream=h.stream())
    specs = [(abi.SHUD_ARR_Y_ELE_GW, 30, 0), (abi.SHUD_ARR_Y_RIV_STG, 60, 0), (abi.SHUD_ARR_QELE_SURF_TOT, 60, 1),
             (abi.SHUD_ARR_QRIV_DOWN, 30, 1), (abi.SHUD_ARR_Q_RECHARGE, 60, 1)]
    ref = []
    sv = ShudSolver(h, y0, SolverControl(reltol=1e-4, abstol=1e-4, init_step=1e-2, max_step=10.0, et_step=60.0))
    h.summary(sv.ode.state_device())
    for k, (arr, itv, flx) in enumerate(specs):
        p, n = h.device_array(arr)
        if not p:                                    # diagnostics materialise on first use
            h.eval(0.0, y0)
            h.refresh_diagnostics()
            p, n = h.device_array(arr)
        out.add(tmp_path / f"dev{k}", p, n, itv, flx)
        ref.append((arr, PrintCtrlPy(tmp_path / f"ref{k}", n, itv, flx)))
    names = {abi.SHUD_ARR_QELE_SURF_TOT: "qele_surf_tot", abi.SHUD_ARR_QRIV_DOWN: "qriv_down",
             abi.SHUD_ARR_Q_RECHARGE: "q_recharge"}

    def cb(i, t, y):
        host = _host_summary(m, y)
        d = h.diagnostics()
        for arr, p in ref:
            p.print_data(host[arr] if arr in host else d[names[arr]], t)

    t, _ = sv.run(12, output=out, on_output=cb)
    assert abs(t - 120.0) < 1e-9
    rows = [out.rows(k) for k in range(len(specs))]
    out.close()
    for _, p in ref:
        p.close()
    assert rows == [4, 2, 2, 4, 2], rows
    for k in range(len(specs)):
        assert open(tmp_path / f"dev{k}.dat", "rb").read() == open(tmp_path / f"ref{k}.dat", "rb").read(), k
    sv.close()
    h.close()


def test_writer_errors_surface(tmp_path):
    """A failing output file (the .dat opened on /dev/full: every write or flush fails with ENOSPC) is
    reported by shud_out_flush and shud_out_destroy instead of being dropped silently; a healthy
    control beside it keeps its rows."""
    m, y0 = cases.ccw()
    m.step = workload.random_step_inputs(m, seed=3)
    h = rt.RhsHandle(m)
    h.set_step_inputs()
    dy, ddy = h.device_alloc(8 * m.num_y), h.device_alloc(8 * m.num_y)
    h.h2d(dy, y0)
    h.eval_device(0.0, dy, ddy)
    h.summary(dy)
    p, n = h.device_array(abi.SHUD_ARR_Y_ELE_SURF)
    (tmp_path / "full.dat").symlink_to("/dev/full")
    out = rt.Output(stream=h.stream())
    out.add(tmp_path / "ok", p, n, 30, 0)
    out.add(tmp_path / "full", p, n, 30, 0)
    for t in (30.0, 60.0, 90.0):
        out.export(t)
    with pytest.raises(rt.ShudRhsError):
        out.flush()
    with pytest.raises(rt.ShudRhsError):
        out.close()
    assert read_dat(tmp_path / "ok.dat")["data"].shape == (3, n)
    h.device_free(dy)
    h.device_free(ddy)
    h.close()
