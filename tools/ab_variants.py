"""A/B the element-kernel build variants on one mesh in one process (interleaved, n rounds).
Every variant must produce bit-identical ydot (same arithmetic, different schedule/placement).
usage: python tools/ab_variants.py [--n-ele N] [--variants 0,1,2,...] [--rounds 3] [--reps 20]
A variant lib:NAME runs the packed kernel of shud-up_amd/build/ab/libshud_rhs_NAME.so (tools/ablib.sh), loaded
beside the production library in the same process, so library builds interleave round by round."""
import argparse
import json
import os
import sys
import time

import ctypes as C

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shud-up_amd"))
from shud_rhs import abi, runtime, synth, workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n-ele", type=int, default=10_000_000)
ap.add_argument("--variants", default="soa,pk",
                help="soa = the SoA kernel (SHUD_RHS_PACKED=0); pk = the packed class-layout kernel; "
                     "pk+NAME=VAL = pk with run-time switches; lib:NAME = an A/B library build")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--ksath-mod", type=int, default=0,
                help="KsatH * (1 + 1e-7 (i %% K)): about 33 K parameter classes (K = 2: the 36..128-class LDS table)")
ap.add_argument("--many-class", action="store_true",
                help="KsatH per element (bench.py many_class: 13,200 tuples -> the hybrid layout)")
a = ap.parse_args()
m = synth.synth_model(a.n_ele)
m.step = workload.random_step_inputs(m)
y = workload.random_state(m)
if a.ksath_mod > 1:
    m.par["KsatH"] = m.par["KsatH"] * (1.0 + 1e-7 * (np.arange(m.num_ele) % a.ksath_mod))
if a.many_class:
    m.par["KsatH"] = m.par["KsatH"] * (1.0 + 1e-7 * (np.arange(m.num_ele) % 400))
vs = a.variants.split(",")


_libs = {}


def lib_for(v):
    """the bound library a variant runs on: production, or an A/B build loaded RTLD_LOCAL beside it"""
    if not v.startswith("lib:"):
        return runtime.lib() if "prod" not in _libs else _libs["prod"]
    name = v[4:].split("+", 1)[0]
    if name not in _libs:
        _libs[name] = abi.bind(C.CDLL(os.path.join(ROOT, "shud-up_amd", "build", "ab", f"libshud_rhs_{name}.so")), strict=False)
    return _libs[name]


def env_for(v):
    # pk+NAME=VAL[+NAME=VAL]: the packed kernel with extra environment (run-time switches, e.g. pk+SHUD_RHS_QD=0)
    if v.startswith("pk+"):
        e = {"SHUD_RHS_PACKED": "1"}
        e.update(kv.split("=", 1) for kv in v[3:].split("+"))
        return e
    if v.startswith("lib:"):     # lib:NAME[+NAME=VAL...]: an A/B library, optionally with run-time switches
        e = {"SHUD_RHS_PACKED": "1"}
        e.update(kv.split("=", 1) for kv in v[4:].split("+")[1:])
        return e
    if v.startswith("soa"):
        return {"SHUD_RHS_PACKED": "0"}
    return {"SHUD_RHS_PACKED": "1"}
res = {v: [] for v in vs}
rres = {v: [] for v in vs}
wres = {v: [] for v in vs}
_saved = {}
ref = None
_libs["prod"] = runtime.lib()
for rnd in range(a.rounds):
    for v in vs:
        for k in _saved:                           # undo the previous variant's extra switches
            os.environ.pop(k, None)
        ev = env_for(v)
        _saved = {k: 1 for k in ev}
        os.environ.update(ev)
        runtime._LIB = lib_for(v)                 # every call of this handle goes to the variant's library
        h = runtime.RhsHandle(m)
        h.set_step_inputs()
        dp, dd = h.device_alloc(8 * m.num_y), h.device_alloc(8 * m.num_y)
        h.h2d(dp, y)
        h.eval_device(0.0, dp, dd)
        out = h.d2h(np.zeros(m.num_y), dd)
        if ref is None:
            ref = out
        same = bool(np.array_equal(out, ref))
        ms, per = h.time_kernels(0.0, dp, dd, a.reps)
        res[v].append(per["shud_ele_kernel"])
        rres[v].append(per["shud_riv_kernel"])
        # event-free: reps back-to-back evals between two synchronizes (what a caller's RHS loop sees)
        h.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            h.eval_device(0.0, dp, dd)
        h.synchronize()
        wres[v].append((time.perf_counter() - t0) / a.reps * 1e3)
        print(f"round {rnd} variant {v:5s} {h.layout()}: ele {per['shud_ele_kernel']:.4f} ms riv {per['shud_riv_kernel']:.4f} "
              f"ms  wall {wres[v][-1]:.4f} ms/eval  bit-identical={same}", flush=True)
        h.device_free(dp); h.device_free(dd); h.close()
        runtime._LIB = _libs["prod"]
print(json.dumps({"num_ele": m.num_ele, "ele_ms_median": {v: float(np.median(t)) for v, t in res.items()},
                  "riv_ms_median": {v: float(np.median(t)) for v, t in rres.items()},
                  "wall_ms_per_eval_median": {v: float(np.median(t)) for v, t in wres.items()}}))
