"""GPU: the device-resident integrator (include/shud_ode.h) against the CPU restatement
(oracle/shud_oracle_ode.c, CVODE 6.0.0 BDF/Newton/SPGMR as SetCVODE configures it).

(1) IEEE-exact test RHS (Robertson, decay, n-component decay over many blocks): with the oracle's reductions in
    the device's fixed order, every output and every counter is bit-identical — the fused device kernels
    perform CVODE's N_Vector arithmetic exactly, and the host control makes the same decisions.
(2) The SHUD RHS (ccw; the branch-variant mesh with the device ET prelude coupled as in SHUD()'s loop): device
    RHS + device integrator vs oracle RHS + oracle integrator.  The RHS itself differs by OCML-vs-glibc ulps, so
    states agree to a small fraction of the solver's own error weight and the step/order sequences match.
    OMP semantics (stateless RHS): the gap stays ~1e-9 of the error weight over 6 simulated hours.  Serial
    semantics: the reference's carried u_satn/qEleE_IC make every RHS call depend on the previous one — including
    the difference-quotient J*v probes — and that feedback amplifies the pow/cbrt ulp differences ~10x per
    10-minute solver step on ccw (tests/diag_ode.py), so serial runs are compared over the first hour only.
    (The model itself is that sensitive: a 1-ulp perturbation of every initial state moves the CPU restatement's
    own ccw trajectory by 3e-2 of the error weight within 10 minutes, in either mode — branchy RHS.)
(3) A physics error inside the integration surfaces as CV_RHSFUNC_FAIL and the reference exit code.
"""
import ctypes as C
import os

import numpy as np
import pytest

import cases
import oracle
from conftest import PKG_DIR, assert_close
from shud_rhs import abi, et
from shud_rhs import runtime as rt
from shud_rhs.solver import ShudSolver, SolverControl

pytestmark = pytest.mark.gpu

COUNTERS = ["nst", "nfe", "nfe_ls", "nni", "ncfn", "nnf", "netf", "nsetups", "nli", "ncfl", "njtimes", "qlast",
            "qcur", "hlast", "hcur", "tcur", "hnext"]


@pytest.fixture(scope="module")
def kat():
    lib = C.CDLL(os.path.join(PKG_DIR, "libshud_kat.so"))
    lib.shud_kat_ode_user.restype = C.c_void_p
    lib.shud_kat_ode_user.argtypes = [C.c_int]
    lib.shud_kat_ode_stream.restype = C.c_void_p
    lib.shud_kat_ode_stream.argtypes = [C.c_void_p]
    lib.shud_kat_ode_set_n.argtypes = [C.c_int64]
    lib.shud_kat_ode_free.argtypes = [C.c_void_p]
    rt.lib()
    return lib


@pytest.fixture
def device_order():
    oracle.OracleOde.set_reduction_order(1)
    yield
    oracle.OracleOde.set_reduction_order(0)


def _dev(kat, problem, n):
    u = kat.shud_kat_ode_user({"robertson": 1, "decay": 2, "decayn": 3}[problem])
    kat.shud_kat_ode_set_n(n)
    fn = C.cast(kat.shud_kat_ode_rhs, C.c_void_p).value
    return u, (fn, u, kat.shud_kat_ode_stream(u))


def _same_stats(a, b):
    for k in COUNTERS:
        assert a[k] == b[k], (k, a[k], b[k])


@pytest.mark.parametrize("problem,n,rtol,atol,h0,touts", [
    ("robertson", 3, 1e-6, 1e-12, 1e-6, [0.4, 4.0, 40.0, 400.0, 4e3, 4e4, 4e5]),
    ("decay", 3, 1e-8, 1e-12, 1e-4, [0.1, 1.0, 5.0]),
    ("decayn", 7 * 40000, 1e-6, 1e-10, 1e-5, [0.01, 1.0, 10.0]),
])
def test_device_integrator_bit_identical(kat, device_order, problem, n, rtol, atol, h0, touts):
    y0 = np.array([1.0, 0.0, 0.0]) if problem == "robertson" else 1.0 + 0.5 * np.sin(np.arange(n))
    u, fn = _dev(kat, problem, n)
    d = rt.OdeSolver(None, 0.0, y0, rtol, atol, h0, 0.0, 0.0, fn=fn)
    o = oracle.OracleOde(problem, 0.0, y0, rtol, atol, h0, 0.0, 0.0)
    for tout in touts:
        fd, td, yd = d.solve(tout)
        fo, to, yo = o.solve(tout)
        assert fd == fo == 0 and td == to == tout
        assert np.array_equal(yd, yo), (tout, np.abs(yd - yo).max())
    _same_stats(d.stats(), o.stats())
    d.close()
    kat.shud_kat_ode_free(u)


def test_device_stop_time_one_step_dky(kat, device_order):
    u, fn = _dev(kat, "decay", 3)
    y0 = np.ones(3)
    d = rt.OdeSolver(None, 0.0, y0, 1e-6, 1e-10, 1e-3, 0.0, 0.0, fn=fn)
    o = oracle.OracleOde("decay", 0.0, y0, 1e-6, 1e-10, 1e-3, 0.0, 0.0)
    for s in (d, o):
        s.set_stop_time(0.25)
    rd, ro = d.solve(1.0), o.solve(1.0)
    assert rd[0] == ro[0] == abi.ODE_TSTOP_RETURN and rd[1] == ro[1] == 0.25 and np.array_equal(rd[2], ro[2])
    for _ in range(5):
        rd, ro = d.solve(1.0, one_step=True), o.solve(1.0, one_step=True)
        assert rd[0] == ro[0] == 0 and rd[1] == ro[1] and np.array_equal(rd[2], ro[2])
    for k in range(3):
        for tt in [rd[1], rd[1] - 0.3 * d.stats()["hlast"]]:
            (fd, dd), (fo, do) = d.get_dky(tt, k), o.get_dky(tt, k)
            assert fd == fo
            if fd == 0:
                assert np.array_equal(dd, do), (k, tt)
    assert d.get_dky(rd[1] + 5.0, 0)[0] == -25
    _same_stats(d.stats(), o.stats())
    d.close()
    kat.shud_kat_ode_free(u)


def test_state_device_complete_for_other_streams(kat, device_order):
    """shud_ode_state_device after lazy one-step solves (no y_out: zn[0]'s completion still deferred on the
    integrator's non-blocking stream): the pointer it returns is read at once by a plain hipMemcpy on the null
    stream and must hold y(tcur) bit for bit (the call now completes and synchronizes)."""
    n = 7 * 40000
    u, fn = _dev(kat, "decayn", n)
    y0 = 1.0 + 0.5 * np.sin(np.arange(n))
    d = rt.OdeSolver(None, 0.0, y0, 1e-6, 1e-10, 1e-5, 0.0, 0.0, fn=fn)
    o = oracle.OracleOde("decayn", 0.0, y0, 1e-6, 1e-10, 1e-5, 0.0, 0.0)
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    for k in range(6):
        d.solve(1.0, one_step=True, y_out=False)
        fo, to, yo = o.solve(1.0, one_step=True)
        ptr = d.state_device()
        assert ptr
        got = np.empty(n)
        assert hip.hipMemcpy(got.ctypes.data, ptr, 8 * n, 2) == 0          # hipMemcpyDeviceToHost, null stream
        assert np.array_equal(got, yo), (k, np.abs(got - yo).max())
    d.close()
    kat.shud_kat_ode_free(u)


def _close_traj(yd, yo, what, frac=1e-6, rtol=1e-4, atol=1e-4):
    """per-state error below `frac` of the solver's own error weight 1/ewt = rtol|y| + atol"""
    err = np.abs(yd - yo)
    tol = frac * (rtol * np.abs(yo) + atol)
    assert np.all(err <= tol), f"{what}: max err {err.max():.3e} at {int(np.argmax(err / tol))}"


@pytest.mark.parametrize("mode,nsteps", [(abi.SHUD_MODE_SERIAL, 6), (abi.SHUD_MODE_OMP, 36)])
def test_shud_ccw_integration_vs_oracle(device_order, mode, nsteps):
    m, y0 = cases.ccw()
    h = rt.RhsHandle(m, mode=mode)
    h.set_step_inputs()
    r = oracle.OracleRhs(m, mode)
    r.set_step_inputs()
    # ccw.cfg.para: ABSTOL 1e-4, RELTOL 1e-4, INIT_SOLVER_STEP 1, MAX_SOLVER_STEP 10; SetCVODE: min step 1e-6
    d = rt.OdeSolver(h, 0.0, y0, 1e-4, 1e-4, 1.0, 10.0, 1e-6, 1000000)
    o = oracle.OracleOde(r, 0.0, y0, 1e-4, 1e-4, 1.0, 10.0, 1e-6, 1000000)
    for k in range(1, nsteps + 1):               # 10-minute solver steps (CV_NORMAL)
        fd, td, yd = d.solve(10.0 * k)
        fo, to, yo = o.solve(10.0 * k)
        assert fd == fo == 0 and td == to
        _close_traj(yd, yo, f"t={td}")
    sd, so = d.stats(), o.stats()
    for key in ["nst", "nfe", "nni", "nli", "netf", "ncfn", "qcur"]:
        assert sd[key] == so[key], (key, sd[key], so[key])
    assert h.num_calls() == sd["nfe"] + sd["nfe_ls"]       # every RHS call went through the device handle
    d.close()
    h.close()


@pytest.mark.parametrize("mode,nsteps", [(abi.SHUD_MODE_SERIAL, 1), (abi.SHUD_MODE_OMP, 2)])
def test_shud_loop_with_device_et_vs_oracle(device_order, mode, nsteps):
    """SHUD()'s loop (shud.cpp:89-131) with ET sub-stepping: per ET step the device prelude writes the step
    inputs in place, then CVode(tout) with CVodeSetStopTime(tout).  The oracle runs the same loop in lockstep;
    its RHS is fed the device prelude's outputs (the prelude's own parity is tests/test_gpu_et.py, checked
    again here), so the comparison isolates integrator + RHS.  ShudSolver, the product driver of this loop,
    must reproduce the hand-driven device run bit for bit."""
    m, y0 = cases.variant(3000, seed=21)
    etm = et.synth_et(m.num_ele, seed=6, terrain=True, lake_frac=0.0)
    ctl = SolverControl(reltol=1e-4, abstol=1e-4, init_step=0.5, max_step=60.0, et_step=20.0)
    assert ctl.et_substep

    def forcing(t, tout):
        return et.synth_forcing(t, tout - t, seed=int(t) + 1, tsr_mode=abi.SHUD_TSR_RECOMPUTE)

    def device_handle():
        h = rt.RhsHandle(m, mode=mode)
        h.set_step_inputs()
        h.et_attach(etm)
        return h

    h = device_handle()
    d = rt.OdeSolver(h, 0.0, y0, ctl.reltol, ctl.abstol, ctl.init_step, ctl.max_step, ctl.min_step,
                     ctl.max_num_steps)
    oe = oracle.OracleEt(etm)
    r = oracle.OracleRhs(m, mode)
    r.set_step_inputs()
    o = oracle.OracleOde(r, 0.0, y0, ctl.reltol, ctl.abstol, ctl.init_step, ctl.max_step, ctl.min_step,
                         ctl.max_num_steps)
    t, tnext, dev_out, k = 0.0, 0.0, [], 0
    for i in range(nsteps):
        tnext += ctl.solver_step
        while t + 1e-10 < tnext:
            tout = min(t + ctl.et_step, tnext)
            f = forcing(t, tout)
            assert h.et_step(f) == abi.SHUD_OK
            assert oe.step(f) == (0, -1)
            got, ref = h.et_get(), oe.get()
            for key in ["qEleNetPrep", "qPotEvap", "qPotTran", "qEleETP", "qEleE_IC"]:
                assert_close(got[key], ref[key], what=f"ET {key} t={t}")
            r.set_step_inputs(step=dict(net_prep=got["qEleNetPrep"], pot_evap=got["qPotEvap"],
                                        pot_tran=got["qPotTran"], etp=got["qEleETP"], lai=got["t_lai"],
                                        fu_surf=got["fu_surf"], fu_sub=got["fu_sub"], e_ic=got["qEleE_IC"]))
            d.set_stop_time(tout)
            o.set_stop_time(tout)
            fd, td, yd = d.solve(tout)
            fo, t, y = o.solve(tout)
            assert fd == fo and fo in (abi.ODE_SUCCESS, abi.ODE_TSTOP_RETURN) and td == t == tout
            # first hour: a 1e-6 fraction of the error weight; later the branchy RHS has amplified the ulp
            # differences (module docstring) and the bound is the solver's own tolerance
            _close_traj(yd, y, f"t={t}", frac=1e-6 if k < 3 else 1.0)
            if k == 2:
                sd, so = d.stats(), o.stats()
                for key in ["nst", "nfe", "nni", "nli", "netf", "ncfn"]:
                    assert sd[key] == so[key], (key, sd[key], so[key])
            k += 1
        dev_out.append(yd)
    sd = d.stats()
    assert h.num_calls() == sd["nfe"] + sd["nfe_ls"]
    d.close()
    h.close()
    # the product driver
    h2 = device_handle()
    sol = ShudSolver(h2, y0, ctl)
    outs = []
    sol.run(nsteps, forcing=forcing, on_output=lambda i, tt, yy: outs.append(yy.copy()))
    for i in range(nsteps):
        assert np.array_equal(outs[i], dev_out[i]), i
    assert sol.stats()["nfe"] == sd["nfe"]
    sol.close()
    h2.close()


def test_physics_error_surfaces():
    m, y0 = cases.ccw()
    y = y0.copy()
    y[5] = np.nan                                   # NaN surface storage: the applyDY NaN check (exit 10)
    h = rt.RhsHandle(m)
    h.set_step_inputs()
    d = rt.OdeSolver(h, 0.0, y, 1e-4, 1e-4, 1.0, 10.0)
    flag, t, _ = d.solve(10.0)
    assert flag == abi.ODE_RHSFUNC_FAIL
    assert h.get_error()["exit_code"] == 10
    d.close()
    h.close()


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_ccw_one_day_trajectory(mode):
    """One simulated day (144 solver steps) of ccw, device chain vs CPU oracle chain (tests/traj.py).

    The chains agree to ~1e-13 of the error weight for the first steps; OCML-vs-glibc ulps in pow/cbrt then grow
    through the carried u_satn / qEleE_IC feedback (serial) until the two runs take different internal step
    sequences and become two independent CVODE solutions of the same problem, whose difference is set by the
    integration tolerance, not by rounding.  The bound is MEASURED, not chosen: traj.spread
    runs the oracle chain against itself with the other reduction order and from initial states one ulp away
    (CPU only, ~20 s), i.e. what rounding-level differences alone do to this problem over the day
    (profiles/r04/traj/spread.json: serial envelope max 13.1 / p95 3.7, OMP 5.9 / 5.8).  Asserted: the device
    chain's max and 95th-percentile weighted difference over the day are within twice that envelope, the first
    hour within 1e-6 of the error weight (tighter than any ulp-perturbed CPU chain reaches), water volume within
    1e-5 relative, both chains finishing every step, step counts within 10 %."""
    import traj
    env = traj.spread(mode)["envelope"]
    rows = traj.run(mode)
    assert len(rows) == 144
    assert all(r["flag_dev"] == r["flag_cpu"] == 0 for r in rows)
    assert max(r["werr"] for r in rows[:6]) <= 1e-6
    werr = np.array([r["werr"] for r in rows])
    assert werr.max() <= 2.0 * env["max"], (werr.max(), env)
    assert np.percentile(werr, 95) <= 2.0 * env["p95"], (np.percentile(werr, 95), env)
    assert max(r["vol_rel"] for r in rows) <= 1e-5
    nd, nc = rows[-1]["nst"]
    assert abs(nd - nc) <= 0.1 * nc
