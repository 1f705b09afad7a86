"""River-order measurement (DESIGN §7.2, round-3 verdict item 4): the same synthetic network under three caller
reach numberings — "band" (the generator's order), "bfs" (breadth-first from the outlets) and "dfs" (depth-first
pre-order: a chain of single reaches contiguous) — one handle each, kernels timed interleaved round by round.
The numbering is the caller's here, so the numbers bound what an internal river-kernel numbering could gain
before it pays the y / DY scatter through a permutation.
usage: python tools/riv_order_ab.py [--n-ele N] [--orders band,dfs,bfs] [--rounds 5] [--reps 20] [--lib NAME ...]
--lib NAME also times the same three handles' kernels on shud-up_amd/build/ab/libshud_rhs_NAME.so (tools/ablib.sh,
e.g. a timing-only SHUD_RIV_ABL build), each handle created on that library."""
import argparse
import json
import os
import sys

import ctypes as C

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shud-up_amd"))
from shud_rhs import abi, runtime, synth, workload  # noqa: E402


def locality(m):
    """per 64-reach wave: downstream / upstream reach records outside the wave's own 64 (means)"""
    d = m.riv_down.astype(np.int64)
    w = np.arange(m.num_riv) // 64
    ok = d >= 0
    src, dst = np.nonzero(ok)[0], d[ok]
    foreign_down = np.unique(np.stack([w[src], dst])[:, w[src] != w[dst]], axis=1)
    foreign_up = np.unique(np.stack([w[dst], src])[:, w[src] != w[dst]], axis=1)
    nw = int(w[-1]) + 1
    return {"foreign_down_per_wave": foreign_down.shape[1] / nw, "foreign_up_per_wave": foreign_up.shape[1] / nw,
            "median_abs_down_minus_r": float(np.median(np.abs(dst - src)))}


ap = argparse.ArgumentParser()
ap.add_argument("--n-ele", type=int, default=10_000_000)
ap.add_argument("--orders", default="band,dfs,bfs")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--lib", action="append", default=[])
a = ap.parse_args()
os.environ.update({"SHUD_RHS_PACKED": "1", "SHUD_RHS_ELE_VARIANT": "0", "SHUD_RHS_SEG_ORDER": "element"})
orders = a.orders.split(",")
prod = runtime.lib()
libs = {"": prod}
for n in a.lib:
    libs[n] = abi.bind(C.CDLL(os.path.join(ROOT, "shud-up_amd", "build", "ab", f"libshud_rhs_{n}.so")))
hs, info = {}, {}
for o in orders:
    m = synth.synth_model(a.n_ele, reach_order=o)
    m.step = workload.random_step_inputs(m)
    y = workload.random_state(m)
    info[o] = locality(m)
    for ln, lb in libs.items():
        runtime._LIB = lb                          # every call of this handle goes to its library
        h = runtime.RhsHandle(m)
        h.set_step_inputs()
        dp, dd = h.device_alloc(8 * m.num_y), h.device_alloc(8 * m.num_y)
        h.h2d(dp, y)
        h.eval_device(0.0, dp, dd)
        hs[(o, ln)] = (h, dp, dd)
        print(o, ln or "prod", m.num_riv, m.num_seg, h.layout(), json.dumps(info[o]), flush=True)
    del m, y
keys = [(o, ln) for o in orders for ln in libs]
tag = lambda k: k[0] + (":" + k[1] if k[1] else "")
ele = {tag(k): [] for k in keys}
riv = {tag(k): [] for k in keys}
for rnd in range(a.rounds):
    for k in keys:
        h, dp, dd = hs[k]
        runtime._LIB = libs[k[1]]
        ms, per = h.time_kernels(0.0, dp, dd, a.reps)
        ele[tag(k)].append(per["shud_ele_kernel"])
        riv[tag(k)].append(per["shud_riv_kernel"])
        print(f"round {rnd} {tag(k):12s}: ele {per['shud_ele_kernel']:.4f} ms riv {per['shud_riv_kernel']:.4f} ms",
              flush=True)
for k in keys:
    h, dp, dd = hs[k]
    runtime._LIB = libs[k[1]]
    h.device_free(dp); h.device_free(dd); h.close()
runtime._LIB = prod
print(json.dumps({"num_ele": a.n_ele, "locality": info,
                  "ele_ms_median": {o: float(np.median(t)) for o, t in ele.items()},
                  "riv_ms_median": {o: float(np.median(t)) for o, t in riv.items()}}))
