"""Long-horizon trajectory agreement: one simulated day of ccw through the device chain (RHS handle + device
integrator) and the CPU oracle chain (oracle RHS + oracle CVODE restatement), 10-minute solver steps as
SHUD()'s loop (shud.cpp:89-140) with ccw.cfg.para's tolerances.  Per step: the error-weighted difference
max_i |y_dev - y_cpu| / (rtol |y_cpu| + atol), the max absolute difference per state block, the total
water volume difference (surface + unsaturated + groundwater, area-weighted) and both solvers' counters.
usage: python tests/diag_traj_day.py [out.json]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "oracle", "shud-up_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    from traj import run
    out = sys.argv[1] if len(sys.argv) > 1 else None
    res = {}
    for mode, name in ((0, "serial"), (1, "omp")):
        rows = run(mode)
        res[name] = rows
        first = next((r["t_min"] for r in rows if r["nst"][0] != r["nst"][1]), None)
        print(f"{name}: max werr {max(r['werr'] for r in rows):.3e}, final werr {rows[-1]['werr']:.3e}, "
              f"max vol_rel {max(r['vol_rel'] for r in rows):.3e}, steps dev/cpu {rows[-1]['nst']}, "
              f"first step-count divergence at t={first}", flush=True)
        for r in rows[:6] + rows[6::12]:
            print(f"  t={r['t_min']:7.1f} werr={r['werr']:.3e} vol_rel={r['vol_rel']:.2e} nst={r['nst']}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
