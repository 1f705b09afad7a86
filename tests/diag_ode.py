"""Diagnostic: device integrator vs CPU restatement on ccw, per solver step (weighted error, counters)."""
import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, "shud-up_amd")
import cases, oracle
from shud_rhs import abi, runtime as rt

oracle.OracleOde.set_reduction_order(1)
for mode in (abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP):
    m, y0 = cases.ccw()
    h = rt.RhsHandle(m, mode=mode); h.set_step_inputs()
    r = oracle.OracleRhs(m, mode); r.set_step_inputs()
    d = rt.OdeSolver(h, 0.0, y0, 1e-4, 1e-4, 1.0, 10.0, 1e-6, 1000000)
    o = oracle.OracleOde(r, 0.0, y0, 1e-4, 1e-4, 1.0, 10.0, 1e-6, 1000000)
    for k in range(1, 37):
        fd, td, yd = d.solve(10.0 * k)
        fo, to, yo = o.solve(10.0 * k)
        w = 1.0 / (1e-4 * np.abs(yo) + 1e-4)
        sd, so = d.stats(), o.stats()
        print(mode, k, fd, fo, f"werr={np.max(np.abs(yd-yo)*w):.3e}", sd["nst"], so["nst"], sd["nfe"], so["nfe"],
              sd["nli"], so["nli"], sd["qcur"], so["qcur"], f"{sd['hcur']:.6f} {so['hcur']:.6f}")
    d.close(); h.close()
