"""Long-horizon trajectory agreement (tests/test_gpu_ode.py::test_ccw_one_day_trajectory, tests/diag_traj_day.py):
one simulated day of ccw through the device chain (RHS handle + device integrator) and the CPU oracle chain
(oracle RHS + oracle CVODE restatement), 10-minute solver steps as SHUD()'s loop (shud.cpp:89-140) with
ccw.cfg.para's tolerances (RELTOL = ABSTOL = 1e-4, INIT_SOLVER_STEP 1, MAX_SOLVER_STEP 10).  Per step: the
error-weighted difference max_i |y_dev - y_cpu| / (rtol |y_cpu| + atol), the max absolute difference per state
block, the relative difference of the total water volume and both solvers' counters."""
import numpy as np


def run(mode, nsteps=144, dt=10.0):
    import cases
    import oracle
    from shud_rhs import runtime as rt
    oracle.OracleOde.set_reduction_order(1)
    m, y0 = cases.ccw()
    NE, NR = m.num_ele, m.num_riv
    h = rt.RhsHandle(m, mode=mode)
    h.set_step_inputs()
    r = oracle.OracleRhs(m, mode)
    r.set_step_inputs()
    d = rt.OdeSolver(h, 0.0, y0, 1e-4, 1e-4, 1.0, 10.0, 1e-6, 1000000)
    o = oracle.OracleOde(r, 0.0, y0, 1e-4, 1e-4, 1.0, 10.0, 1e-6, 1000000)
    area = m.ele["area"]
    sy = m.par["Sy"]
    rows = []
    for k in range(1, nsteps + 1):
        fd, td, yd = d.solve(dt * k)
        fo, to, yo = o.solve(dt * k)
        w = 1.0 / (1e-4 * np.abs(yo) + 1e-4)
        diff = np.abs(yd - yo)
        vol = lambda y: float(np.sum(area * (y[:NE] + y[NE:2 * NE] * sy + y[2 * NE:3 * NE] * sy)))
        sd, so = d.stats(), o.stats()
        rows.append({"t_min": td, "flag_dev": fd, "flag_cpu": fo, "werr": float(np.max(diff * w)),
                     "max_abs": {"sf": float(diff[:NE].max()), "us": float(diff[NE:2 * NE].max()),
                                 "gw": float(diff[2 * NE:3 * NE].max()), "riv": float(diff[3 * NE:].max())},
                     "vol_rel": abs(vol(yd) - vol(yo)) / abs(vol(yo)),
                     "nst": [sd["nst"], so["nst"]], "nfe": [sd["nfe"] + sd["nfe_ls"], so["nfe"] + so["nfe_ls"]]})
    d.close()
    h.close()
    return rows
