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


def _cpu_chain(mode, order, y0, nsteps, dt):
    import cases
    import oracle
    oracle.OracleOde.set_reduction_order(order)
    m, _ = cases.ccw()
    r = oracle.OracleRhs(m, mode)
    r.set_step_inputs()
    o = oracle.OracleOde(r, 0.0, y0, 1e-4, 1e-4, 1.0, 10.0, 1e-6, 1000000)
    out = [o.solve(dt * k)[2].copy() for k in range(1, nsteps + 1)]
    nst = o.stats()["nst"]
    oracle.OracleOde.set_reduction_order(1)
    return out, nst


def spread(mode, nsteps=144, dt=10.0):
    """The problem's own divergence over the day, CPU only: the oracle chain (device reduction
    order) against itself run with the other reduction order, and from initial states moved by one ulp (all entries
    up, all down, three random-sign patterns).  Per variant: max / 95th percentile of the error-weighted difference
    over the day.  The envelope (max over the variants) is what rounding-level differences alone produce; the
    device-vs-oracle trajectory test bounds the device chain by twice it."""
    import cases
    _, y0 = cases.ccw()
    ref, nref = _cpu_chain(mode, 1, y0, nsteps, dt)
    variants = {"order0": (0, y0), "ulp_up": (1, np.nextafter(y0, np.inf)), "ulp_down": (1, np.nextafter(y0, -np.inf))}
    for s in (1, 2, 3):
        rng = np.random.default_rng(s)
        variants[f"ulp_rand{s}"] = (1, np.where(rng.random(y0.size) < 0.5, np.nextafter(y0, np.inf),
                                                np.nextafter(y0, -np.inf)))
    out = {}
    for name, (order, yy) in variants.items():
        b, nb = _cpu_chain(mode, order, yy, nsteps, dt)
        w = np.array([float(np.max(np.abs(x - y) / (1e-4 * np.abs(x) + 1e-4))) for x, y in zip(ref, b)])
        out[name] = {"max": float(w.max()), "p95": float(np.percentile(w, 95)), "nst": [int(nref), int(nb)]}
    out["envelope"] = {"max": max(v["max"] for v in out.values()), "p95": max(v["p95"] for v in out.values())}
    return out
