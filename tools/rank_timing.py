"""Per-rank RHS time of the N > 1 decomposition, measured on one GPU (the pool's boxes have one): syn-10M split
by the bench's own C++ partition (PART_AUTO, seed 12345) into N parts; each rank's partitioned handle runs its
eval pipeline (pack kernel, interior elements, boundary + ghost elements, reaches) back to back on the GPU with
the halo already in place (external transport: no RCCL), timed by the in-loop HIP events.  The slowest rank's
time is the compute part of an N-GPU RHS; the RCCL exchange (~100 KB per rank, overlapped with the interior
elements) comes on top.  usage: python tools/rank_timing.py [N ...]  (default 2 4 8) -> one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shud-up_amd"))


def main():
    from shud_rhs import partition, synth, workload
    from shud_rhs import runtime as rt
    ns = [int(a) for a in sys.argv[1:]] or [2, 4, 8]
    t0 = time.time()
    m = synth.synth_model(10_000_000)
    m.step = workload.random_step_inputs(m)
    y = workload.random_state(m)
    print(f"[rank_timing] mesh NE={m.num_ele} in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    out = {"workload": "syn-10M RHS, per-rank partitioned handles on one GPU (halo pre-placed, no RCCL)",
           "num_ele": m.num_ele, "ranks": {}}
    steps, warm = 50, 10
    for n in ns:
        ep, st = partition.cpp_partition(m, n, partition.PART_AUTO, seed=12345)
        rows = []
        for r in range(n):
            pl = partition.CppPlan(m, ep, n, r)
            lm, part = pl.local_model()
            pl.close()
            h = rt.RhsHandle(lm, partition=part)
            h.set_step_inputs()
            yl = partition.local_state(y, m, part)
            dy_ = h.device_alloc(8 * yl.size)
            ddy = h.device_alloc(8 * yl.size)
            h.h2d(dy_, yl)
            gele, griv = partition.ghost_values(y, m, part)
            _, _, d_gele, d_griv = h.halo_buffers()
            if gele.size:
                h.h2d(d_gele, gele)
            if griv.size:
                h.h2d(d_griv, griv)
            for _ in range(warm):
                h.eval_device(0.0, dy_, ddy)
            h.synchronize()
            h.timing(steps, 1)
            tw = time.perf_counter()
            for _ in range(steps):
                h.eval_device(0.0, dy_, ddy)
            h.synchronize()
            wall = (time.perf_counter() - tw) / steps * 1e3
            ms_ele, ms_riv, ms_eval, nt = h.timing_read()
            tw = time.perf_counter()               # the same pipeline with no timing events in it
            for _ in range(4 * steps):
                h.eval_device(0.0, dy_, ddy)
            h.synchronize()
            wall_untimed = (time.perf_counter() - tw) / (4 * steps) * 1e3
            rows.append({"rank": r, "own_ele": part.n_own_ele, "ghost_ele": lm.num_ele - part.n_own_ele,
                         "own_riv": part.n_own_riv, "layout": h.layout(), "ms_eval": ms_eval, "ms_ele": ms_ele,
                         "ms_riv": ms_riv, "ms_wall_per_eval": wall,
                         "ms_wall_untimed": wall_untimed})
            h.device_free(dy_)
            h.device_free(ddy)
            h.close()
            print(f"[rank_timing] N={n} rank {r}: {rows[-1]}", file=sys.stderr, flush=True)
        slow = max(x["ms_eval"] for x in rows)
        slow_wall = max(x["ms_wall_untimed"] for x in rows)
        out["ranks"][str(n)] = {"partition": {k: st[k] for k in ("method_used", "edge_cut", "segment_cut",
                                                                   "max_halo", "imbalance")},
                                "max_rank_ms_eval": slow, "max_rank_ms_wall_untimed": slow_wall, "projected_value_compute_only": m.num_ele / (slow * 1e-3),
                                "per_rank": rows}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
