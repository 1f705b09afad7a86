"""Timing-only ablations of the river kernel on syn-10M: one process per library, the production one and the
ablation builds of tools/riv_abl.sh (-DSHUD_RIV_ABL bits: 1 no upstream reaches, 2 no segment gathers, 4 no
downstream reach; results are wrong by design).  HIP-event kernel times; run under rocprofv3 --pmc to split
FETCH_SIZE by variant (the ABL template argument is in the kernel name).
usage: [SHUD_RHS_LIB=...] python tools/riv_abl.py [n_ele] [label]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shud-up_amd"))


def main():
    import torch
    from shud_rhs import runtime, synth, workload
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(os.environ.get("SHUD_RHS_LIB", "prod"))
    gm = synth.synth_model(n)
    gm.step = workload.random_step_inputs(gm)
    y = workload.random_state(gm)
    h = runtime.RhsHandle(gm, device=0, stream=torch.cuda.current_stream().cuda_stream)
    h.set_step_inputs()
    yt = torch.from_numpy(y).cuda()
    dt = torch.empty_like(yt)
    for _ in range(3):
        h.eval_device(0.0, yt.data_ptr(), dt.data_ptr())
    h.timing(40, 1)
    for _ in range(40):
        h.eval_device(0.0, yt.data_ptr(), dt.data_ptr())
    me, mr, mv, k = h.timing_read()
    print(f"{label}: riv {mr * 1e3:.1f} us  ele {me * 1e3:.1f} us  ({k} evals)", flush=True)
    h.close()


if __name__ == "__main__":
    main()
