"""debug: the device loop of tests/test_gpu_ode.py::test_shud_loop_with_device_et_vs_oracle, with error reports"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "oracle", "shud-up_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import cases
from shud_rhs import abi, et, runtime as rt
from shud_rhs.solver import SolverControl

for packed in ("1", "0"):
    os.environ["SHUD_RHS_PACKED"] = packed
    m, y0 = cases.variant(3000, seed=21)
    etm = et.synth_et(m.num_ele, seed=6, terrain=True, lake_frac=0.0)
    ctl = SolverControl(reltol=1e-4, abstol=1e-4, init_step=0.5, max_step=60.0, et_step=20.0)
    h = rt.RhsHandle(m, mode=0)
    h.set_step_inputs()
    h.et_attach(etm)
    d = rt.OdeSolver(h, 0.0, y0, ctl.reltol, ctl.abstol, ctl.init_step, ctl.max_step, ctl.min_step, ctl.max_num_steps)
    t = 0.0
    for k in range(3):
        tout = t + ctl.et_step
        f = et.synth_forcing(t, tout - t, seed=int(t) + 1, tsr_mode=abi.SHUD_TSR_RECOMPUTE)
        print("et", h.et_step(f), flush=True)
        d.set_stop_time(tout)
        fd, td, yd = d.solve(tout)
        print("packed", packed, "k", k, "flag", fd, td, h.get_error(), rt.lib().shud_rhs_last_error_string(), flush=True)
        if fd < 0:
            break
        t = tout
    # a plain eval of y0 vs oracle
    import oracle
    h2 = rt.RhsHandle(m, mode=0); h2.set_step_inputs()
    o = oracle.OracleRhs(m, 0); o.set_step_inputs()
    g = h2.eval(0.0, y0); r = o.eval(0.0, y0)[0]
    print("plain eval max diff", np.max(np.abs(g - r)), flush=True)
