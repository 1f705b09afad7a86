"""Element-kernel time vs number of parameter classes on syn-10M (KsatH perturbed by element mod M, 33 x M
classes): the default dispatch (LDS class table: 256-thread workgroups up to 128 classes, 1024-thread workgroups
up to 600, SoA above), the packed layout with the class table read from L2 (SHUD_RHS_L2_CLASS=1) and the SoA
layout, to place the layout switches (shud_rhs.cpp build_packed).  Prints one line per (M, path)."""
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shud-up_amd"))


def main():
    import torch
    from shud_rhs import runtime, synth, workload
    gm = synth.synth_model(10_000_000)
    gm.step = workload.random_step_inputs(gm)
    y = torch.from_numpy(workload.random_state(gm)).cuda()
    dy = torch.empty_like(y)
    base = gm.par["KsatH"]
    for M in (1, 4, 8, 15, 18, 60):
        m2 = copy.copy(gm)
        m2.par = dict(gm.par)
        m2.par["KsatH"] = base * (1.0 + 1e-7 * (np.arange(gm.num_ele) % M))
        for path in ("auto", "l2", "soa"):
            os.environ["SHUD_RHS_L2_CLASS"] = {"auto": "", "l2": "1", "soa": "0"}[path]
            os.environ["SHUD_RHS_PACKED"] = "0" if path == "soa" else "1"
            h = runtime.RhsHandle(m2, device=0, stream=torch.cuda.current_stream().cuda_stream)
            h.set_step_inputs()
            lay = h.layout()
            for _ in range(5):
                h.eval_device(0.0, y.data_ptr(), dy.data_ptr())
            h.timing(30, 1)
            for _ in range(30):
                h.eval_device(0.0, y.data_ptr(), dy.data_ptr())
            me, mr, mv, n = h.timing_read()
            h.close()
            print(f"M={M:4d} path={path:4s} classes={lay['n_classes'] if lay['packed'] else '-':>6} "
                  f"layout={'packed' if lay['packed'] else 'soa':6s} "
                  f"ele {me:.4f} ms  riv {mr:.4f} ms", flush=True)
    os.environ.pop("SHUD_RHS_L2_CLASS")
    os.environ.pop("SHUD_RHS_PACKED")


if __name__ == "__main__":
    main()
