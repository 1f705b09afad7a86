#!/usr/bin/env python3
"""bench.py — SHUD RHS flux assembly on MI355X: element-flux-updates/s (RHS evals x NumEle).

Workload (BASELINE.json north_star / SURVEY §8d): synthetic 10M-triangle mesh (syn-10M: 3162 x 1582 quads,
ccw-like river density, seed 12345), seeded random state y and ET-step inputs, serial (reference `make
shud`) semantics.  One "step" = one RHS evaluation f(t, y, ydot) with y / ydot resident in HBM.
N = 1: the whole mesh on one GPU.  N > 1 (one process per GPU: under torch.distributed.run, or — `--gpus N`
without a launcher — started by bench.py itself before any GPU call, see launch_ranks): the same 10M mesh
partitioned by the C++ partitioner (multilevel or RCB, whichever gives the smaller largest halo) across the N ranks, ghost states exchanged by RCCL (grouped send/recv over xGMI) inside
every RHS call; value = NumEle_total x K / max-over-ranks time ("scaling": "strong": the 10M mesh is fixed).

At N > 1 (and with --partition-1) every rank's DY is then checked bit for bit against a full-mesh single-GPU
handle on its own device (`parity_vs_1gpu`); a fatal error flag on any rank (incl. a timed-out halo poll) or a
parity miss ends the run with a non-zero status and no result line.

Prints ONE JSON line on rank 0 with roofline (dominant kernel: shud_ele_kernel, HIP-event timed on the
stream it runs on) and cpu_baseline (the CPU restatement oracle on this host's cores, bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "shud-up_amd"))

HBM_PEAK = 8.0e12          # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP64_VALU_NOMINAL = 78.6e12   # FLOP/s, MI355X fp64 vector: 256 CUs x 64 fp64 FMA lanes x 2 FLOP x 2.4 GHz max clock
METRIC = "element-flux-updates/sec (RHS evals × NumEle) at 1/2/4/8 GPUs; %HBM roofline"
# algorithmic bytes per RHS (canonical): 392 B/element + 24 B/segment + 96 B/reach
B_ELE, B_SEG, B_RIV = 392, 24, 96


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def shared_partition(gm, world, rank, dist=None, device="cpu"):
    """The N > 1 element partition: rank 0 runs the C++ partitioner (PART_AUTO, seed 12345; deterministic, so
    any rank would get the same parts) and broadcasts the element -> part map and its stats over `dist`."""
    import torch
    from shud_rhs import partition
    if rank == 0:
        ele_part, pst = partition.cpp_partition(gm, world, partition.PART_AUTO, seed=12345)
    else:
        ele_part, pst = np.zeros(gm.num_ele, np.int32), None
    if world > 1 and dist is not None:
        t = torch.from_numpy(ele_part).to(device)
        dist.broadcast(t, src=0)
        ele_part = t.cpu().numpy()
        box = [pst]
        dist.broadcast_object_list(box, src=0)
        pst = box[0]
    return ele_part, pst


FATAL_FLAGS = 0x01 | 0x02 | 0x04 | 0x08 | 0x80   # SHUD_EF_NAN_QELE | EFFKH | ET_NEG | ET_NAN | HALO_WAIT (shud_rhs.h)


# ---- phase heartbeats and watchdogs (the first N > 1 run must end in a number or a named failure) -------------
# Every rank announces each phase on stderr ("[bench-hb] rank R phase P bound B") and, at N > 1, arms a C-level
# watchdog (faulthandler: its own thread, no GIL needed, so it fires inside a stuck RCCL / HIP / c10d call too)
# that dumps every thread's stack and exits the rank with status 1 once the phase outlives its bound.  Under
# torch.distributed.run that ends the job (the agent stops the other ranks); under bench.py's own launcher the
# parent also tracks every rank's last phase and enforces the bound plus a grace period itself, terminating all
# ranks and naming the stuck rank and phase.  Bounds: generous (a fresh box's first `import torch` can take 1-2
# min), scaled by SHUD_BENCH_PHASE_SCALE (tests).
PHASE_BOUND_S = {"start": 420, "init": 240, "mesh": 300, "partition": 360, "handle": 240, "settle": 180,
                 "timed": 180, "parity": 360, "report": 120, "side": 900, "dry_hang": 60}
HB_TAG = "[bench-hb]"


def phase_bound(phase):
    return PHASE_BOUND_S.get(phase, 300) * float(os.environ.get("SHUD_BENCH_PHASE_SCALE", "1"))


def heartbeat(phase, rank, arm):
    """announce `phase` on stderr; with arm, (re)arm the in-rank watchdog for this phase's bound"""
    b = phase_bound(phase)
    print(f"{HB_TAG} rank {rank} phase {phase} bound {b:g}", file=sys.stderr, flush=True)
    if arm:
        import faulthandler
        faulthandler.dump_traceback_later(b, exit=True, file=sys.stderr)


def launch_ranks(nproc, argv, dry):
    """`--gpus N > 1` without a launcher: start the N rank processes here (one per GPU, RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment, rendezvous on 127.0.0.1) BEFORE anything touches the GPU, forward
    the ranks' stdout (rank 0's JSON line) and stderr, and exit with the first non-zero rank status (the others are
    then terminated), naming the rank and the phase it was in.  A watchdog ends the launch when a rank stays in one
    phase longer than its bound + SHUD_BENCH_GRACE_S (default 60 s): every rank is terminated (SIGTERM, SIGKILL
    10 s later) and the launch exits 124.  This process never initialises HIP."""
    import signal
    import socket
    import subprocess
    import threading
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    grace = float(os.environ.get("SHUD_BENCH_GRACE_S", "60"))
    procs, outs = [], []
    phase = [("start", time.monotonic())] * nproc
    lock = threading.Lock()
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SHUD_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        outs.append([])

    def pump_out(k):
        for line in procs[k].stdout:
            outs[k].append(line)

    def pump_err(k):
        for line in procs[k].stderr:
            if line.startswith(HB_TAG):
                f = line.split()
                with lock:
                    phase[k] = (f[4], time.monotonic())
            sys.stderr.write(line)
            sys.stderr.flush()
    th = [threading.Thread(target=fn, args=(k,), daemon=True) for k in range(nproc) for fn in (pump_out, pump_err)]
    for t in th:
        t.start()

    def stop_all(live):
        for j in live:
            procs[j].send_signal(signal.SIGTERM)
        t_end = time.monotonic() + 10
        for j in live:
            try:
                procs[j].wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                procs[j].kill()
                procs[j].wait()

    rc = 0
    live = set(range(nproc))
    while live:
        for k in sorted(live):
            st = procs[k].poll()
            if st is None:
                continue
            live.discard(k)
            if st != 0 and rc == 0:
                rc = st if st > 0 else 128 - st
                with lock:
                    ph = phase[k][0]
                print(f"[bench] rank {k} exited with status {st} in phase {ph!r}: stopping the other ranks",
                      file=sys.stderr, flush=True)
                stop_all(sorted(live))
        if rc == 0 and live:
            now = time.monotonic()
            with lock:
                late = [(k, phase[k][0], now - phase[k][1]) for k in sorted(live)
                        if now - phase[k][1] > phase_bound(phase[k][0]) + grace]
            if late:
                k, ph, el = late[0]
                print(f"[bench] watchdog: rank {k} stuck in phase {ph!r} for {el:.0f} s (bound "
                      f"{phase_bound(ph):g} s + {grace:g} s grace); terminating all {nproc} ranks "
                      f"(last phases: {', '.join(f'rank {j}: {phase[j][0]}' for j in range(nproc))})",
                      file=sys.stderr, flush=True)
                stop_all(sorted(live))
                live.clear()
                rc = 124
        time.sleep(0.05)
    for t in th:
        t.join(timeout=5)
    for k in range(nproc) if dry else [0]:
        sys.stdout.write("".join(outs[k]))
    sys.stdout.flush()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle", type=int, default=200,
                    help="untimed RHS evals before the warm-up: a cold GPU's clocks wander for ~20 ms of load "
                         "(element kernel 0.60 -> 0.65 -> 0.60 ms, profiles/r02/kt); same count on every rank")
    ap.add_argument("--n-ele", type=int, default=10_000_000)
    ap.add_argument("--mode", choices=["serial", "omp"], default="serial")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-reps", type=int, default=20, help="N>1: serialized per-phase timing reps")
    ap.add_argument("--no-host-vectors", action="store_true", help="skip the PCIe-inclusive host-vector eval")
    ap.add_argument("--no-many-class", action="store_true",
                    help="skip the many-parameter-class workloads (L2 class table, SoA fallback)")
    ap.add_argument("--no-et", action="store_true", help="skip the ET-step prelude timing (SURVEY f1)")
    ap.add_argument("--no-ode", action="store_true", help="skip the device integrator timing (SURVEY f2)")
    ap.add_argument("--e2e-ele", type=int, default=100_000,
                    help="elements of the end-to-end shud_gpu run (C++ host, one simulated day); 0 = skip")
    ap.add_argument("--partition-1", action="store_true",
                    help="run the N>1 code path (partitioned handle, RCCL comm, overlap) with one rank (smoke test)")
    ap.add_argument("--no-parity", action="store_true",
                    help="N>1 / --partition-1: skip the bit-identity check of every rank's DY against a full-mesh "
                         "single-GPU handle")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launcher test: each rank reports RANK / WORLD_SIZE and exits before touching the GPU")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.dry_launch))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr, flush=True)
        sys.exit(2)
    # the in-rank watchdog: on at N > 1 (SHUD_BENCH_RANK_WATCHDOG=0 leaves only the launcher's, tests), off at N = 1
    arm = world > 1 and os.environ.get("SHUD_BENCH_RANK_WATCHDOG", "1") != "0"
    hb = lambda phase: heartbeat(phase, rank, arm)            # noqa: E731
    hb("start")
    if args.dry_launch:
        print(json.dumps({"dry_launch": True, "rank": rank, "world_size": world, "local_rank": local,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        if os.environ.get("SHUD_BENCH_DRY_FAIL_RANK") == str(rank):    # launcher test: a failing rank
            sys.exit(5)
        if os.environ.get("SHUD_BENCH_DRY_HANG_RANK") == str(rank):    # launcher test: a rank that never returns
            hb("dry_hang")
            while True:
                time.sleep(1)
        if arm:
            import faulthandler
            faulthandler.cancel_dump_traceback_later()
        return
    # stdout carries exactly one JSON line: libraries that print banners on it (RCCL prints its version block
    # at communicator init) write to stderr instead until the line is printed
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist
    from shud_rhs import abi, partition, runtime, synth, workload

    hb("init")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    mode = abi.SHUD_MODE_SERIAL if args.mode == "serial" else abi.SHUD_MODE_OMP

    hb("mesh")
    t0 = time.time()
    gm = synth.synth_model(args.n_ele)
    gm.step = workload.random_step_inputs(gm)
    y_glob = workload.random_state(gm)
    NE, NR, NS = gm.num_ele, gm.num_riv, gm.num_seg
    log(f"[bench] syn mesh NE={NE} NR={NR} NS={NS} built in {time.time() - t0:.1f}s")

    stream = torch.cuda.current_stream()
    if world > 1 or args.partition_1:
        # the C++ partitioner + planner (include/shud_partition.h): multilevel and RCB, the smaller largest
        # halo wins; rank 0 partitions (deterministic: any rank would get the same parts) and broadcasts the
        # element -> part map, then every rank builds only its own plan
        hb("partition")
        tp = time.time()
        ele_part, pst = shared_partition(gm, world, rank, dist if world > 1 else None, f"cuda:{local}")
        cut_e, cut_s = pst["edge_cut"], pst["segment_cut"]
        plan = partition.CppPlan(gm, ele_part, world, rank)
        lm, part = plan.local_model()
        plan.close()
        log(f"[bench] C++ partition ({'multilevel' if pst['method_used'] == 0 else 'RCB'}, "
            f"{pst['seconds']:.1f}s) + plan/local mesh in {time.time() - tp:.1f}s; largest halo "
            f"{pst['max_halo']} entities")
        uid = [runtime.nccl_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        part.nccl_unique_id = uid[0]
        hb("handle")                       # ncclCommInitRank inside
        h = runtime.RhsHandle(lm, mode=mode, device=local, stream=stream.cuda_stream, partition=part)
        y_loc = partition.local_state(y_glob, gm, part)
        model = lm
        log(f"[bench] {world}-way: edge cut {cut_e} mesh edges, {cut_s} river segments; rank0 "
            f"own {part.n_own_ele} ele / {part.n_own_riv} riv, "
            f"ghosts {lm.num_ele - part.n_own_ele} ele / {lm.num_riv - part.n_own_riv} riv")
    else:
        h = runtime.RhsHandle(gm, mode=mode, device=local, stream=stream.cuda_stream)
        y_loc = y_glob
        model = gm
    h.set_step_inputs()
    y_t = torch.from_numpy(y_loc).to(f"cuda:{local}")
    dy_t = torch.empty_like(y_t)
    yp, dyp = y_t.data_ptr(), dy_t.data_ptr()

    # the STREAM probes (~50 ms of full-bandwidth traffic) run before the warm-up: the clock transient a cold
    # GPU goes through in its first ~20 ms of load (element kernel 0.62 -> 0.74 -> 0.62 ms, profiles/r02/kt) then
    # falls outside the K timed evals instead of inside a short K = 20 window
    sp = stream_probe(local) if world == 1 else {}
    vp = valu_probe(local) if world == 1 else {}
    hb("settle")
    ts = time.perf_counter()
    for _ in range(args.settle):
        h.eval_device(0.0, yp, dyp)
    torch.cuda.synchronize()
    settle_s = time.perf_counter() - ts
    for _ in range(args.warmup):
        h.eval_device(0.0, yp, dyp)
    torch.cuda.synchronize()
    # HIP events around the kernels of every 2nd timed eval (handle's stream = torch's current stream): an event
    # between two kernels stops their tails overlapping (~1 % of an eval), so only a sample of the K evals
    # carries them.  A partitioned rank's eval is ~0.09 ms, where three event records cost ~15 % of the eval
    # (tools/rank_timing.py: 0.105 ms with events on every eval vs 0.089 without), so N > 1 samples 1 in 4
    t_stride = (4 if (world > 1 or args.partition_1) else 2) if args.steps >= 10 else 1
    h.timing(args.steps, t_stride)
    hb("timed")
    # the K timed evals, bracketed by a barrier + synchronize.  Each rank also brackets them with HIP events on its
    # compute stream (torch's current stream = the handle's stream; every eval's last kernel runs there after its
    # halo arrived): at N > 1 the value is timed from the slowest rank's event span, so the trailing barrier (and
    # the ranks' skew leaving it) stays outside the measured window; the barrier-inclusive wall time is reported
    # beside it.  N = 1: the wall time between the two synchronizes.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    ev0.record()
    for k in range(args.steps):
        h.eval_device(0.0, yp, dyp)
    ev1.record()
    torch.cuda.synchronize()
    dt_rank_wall = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt_wall = time.perf_counter() - t_start
    dt_ev = ev0.elapsed_time(ev1) * 1e-3
    dt = dt_wall
    ms_ele_loop, ms_riv_loop, ms_eval_loop, n_timed = h.timing_read()
    kmax = None
    timing_detail = None
    if world > 1:
        tt = torch.tensor([dt_ev, dt_rank_wall, dt_wall], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])
        timing_detail = {"source": "max over ranks of each rank's HIP-event span of the K evals on its compute stream",
                         "ms_per_step_events_max": float(tt[0]) / args.steps * 1e3,
                         "ms_per_step_rank_wall_max": float(tt[1]) / args.steps * 1e3,
                         "ms_per_step_wall_incl_barrier": float(tt[2]) / args.steps * 1e3,
                         "value_wall_incl_barrier": NE * args.steps / float(tt[2]),
                         "note": "value = NumEle x K / the slowest rank's event span (since round 5); rounds 1-4 "
                                 "quoted the barrier-inclusive wall window (value_wall_incl_barrier), which also "
                                 "holds the trailing barrier and the ranks' skew leaving it"}
        # the slowest rank's in-loop kernel times (each rank's HIP events on its own compute stream)
        kt = torch.tensor([ms_ele_loop, ms_riv_loop, ms_eval_loop], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(kt, op=dist.ReduceOp.MAX)
        kmax = {"shud_ele_kernel": float(kt[0]), "shud_riv_kernel": float(kt[1]), "eval": float(kt[2])}
    hb("report")
    # a fatal error flag (NaN fluxes, effKH range, ET checks, a timed-out halo poll) means the timed evals computed
    # wrong DY: no throughput line, non-zero exit on every rank
    err = h.get_error()
    fatal = int(err["flags"]) & FATAL_FLAGS
    if world > 1:
        tf = torch.tensor([fatal], dtype=torch.int64, device=f"cuda:{local}")
        dist.all_reduce(tf, op=dist.ReduceOp.MAX)
        fatal = int(tf.item())
    if fatal:
        print(f"[bench] rank {rank}: fatal error flags 0x{fatal:x} (this rank: {err}) — no result", file=sys.stderr,
              flush=True)
        sys.exit(3)
    parity = None
    if (world > 1 or args.partition_1) and not args.no_parity:
        hb("parity")
        parity = parity_vs_1gpu(h, gm, y_glob, part, mode, local, stream, yp, dyp, dy_t, dist if world > 1 else None)
        if not parity["ok"]:
            print(f"[bench] rank {rank}: DY differs from the single-GPU handle: {parity}", file=sys.stderr, flush=True)
        hb("report")

    # per-kernel times: HIP events recorded inside the timed loop on the handle's stream (= torch's current
    # stream); a partitioned handle also gets a serialized per-phase breakdown (halo exchange alone)
    per = {"shud_ele_kernel": ms_ele_loop, "shud_riv_kernel": ms_riv_loop}
    ms_eval = ms_eval_loop
    if world > 1 and args.profile_reps > 0:
        _, per_ser = h.time_kernels(0.0, yp, dyp, args.profile_reps)
        # pack + grouped send/recv alone (serialized, no overlap), slowest rank
        th = torch.tensor([float(per_ser.get("halo_exchange") or 0.0)], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(th, op=dist.ReduceOp.MAX)
        per["halo_exchange_serialized"] = float(th.item())
        dist.barrier()
    ms_ele = per["shud_ele_kernel"]
    ms_riv = per["shud_riv_kernel"]
    n_own_e = model.num_ele if world == 1 else part.n_own_ele
    n_own_r = model.num_riv if world == 1 else part.n_own_riv
    n_seg_local = model.num_seg
    ele_bytes = B_ELE * n_own_e + B_SEG * n_seg_local
    riv_bytes = B_RIV * n_own_r
    achieved = ele_bytes / (ms_ele * 1e-3)

    value = NE * args.steps / dt
    ms_step = dt / args.steps * 1e3
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "element-flux-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle": {"evals": args.settle, "seconds": round(settle_s, 3),
                   "note": "untimed evals before the warm-up (clock settle), outside the timed region"},
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded jittered-grid Delaunay mesh + river tree, random y and ET-step inputs)",
        "config": {"workload": f"syn-10M RHS ({args.mode} semantics)" if NE >= 9_000_000 else f"syn-{NE} RHS",
                   "num_ele": NE, "num_riv": NR, "num_seg": NS,
                   "parallelism": (f"mesh-partition x{world} (C++ {'multilevel' if pst['method_used'] == 0 else 'RCB'}"
                                   f" partition, RCCL halo)") if world > 1 else "single GPU",
                   **({"edge_cut": cut_e, "segment_cut": cut_s, "max_halo_entities": pst["max_halo"],
                       "imbalance": pst["imbalance"]} if world > 1 else {}),
                   "y_ydot": "device-resident", "kernel_layout": h.layout()},
        "roofline": {
            "bound": "hbm",
            "kernel": "shud_ele_kernel",
            "achieved": achieved / 1e9,
            "peak": HBM_PEAK / 1e9,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK,
            "traffic": None,
            "algorithmic_bytes_per_launch": ele_bytes,
            "frac_note": ("achieved / frac price SURVEY §8d's canonical 392 B per element, which counts every edge's "
                          "neighbour gathers as HBM reads (L2 hits in practice; shared in-tile edges gather nothing), "
                          "so frac can exceed 1; traffic / frac_actual are the PMC-measured bytes"),
            "kernel_ms": {k: v for k, v in per.items()},
            "kernel_ms_source": (f"HIP events around the kernels of {n_timed} of the {args.steps} timed evals "
                                 f"(1 in {t_stride}; handle stream)"),
            **({"kernel_ms_max_over_ranks": kmax} if kmax else {}),
            "rhs_frac": (ele_bytes + riv_bytes) / (ms_eval * 1e-3) / HBM_PEAK,
            "riv_algorithmic_bytes_per_launch": riv_bytes,
            "riv_frac": riv_bytes / (ms_riv * 1e-3) / HBM_PEAK if ms_riv > 0 else None,
        },
        "cpu_baseline": None,
    }
    if timing_detail:
        out["timing"] = timing_detail
    if world > 1 or args.partition_1:
        out["rccl_ranks"] = world
        out["parity_vs_1gpu"] = None if parity is None else parity["all_ok"]
        if parity is not None:
            out["parity_detail"] = {k: parity[k] for k in ("calls", "words_checked_rank0", "ranks_ok", "note")}
        if parity is not None and not parity["all_ok"]:
            sys.stdout.flush()
            print(json.dumps(out), file=sys.stderr, flush=True)
            sys.exit(4)
    # the practical HBM ceilings on this box (measured before the warm-up, see there)
    if sp:
        out["roofline"].update(sp)
        out["roofline"]["frac_of_stream_copy"] = achieved / 1e9 / sp["stream_copy_GBs"]
    # what kind of box this line ran on: its HBM ceilings (STREAM) and its fp64 VALU rate + in-kernel clock under a
    # dense fp64 load; the element kernel is co-limited by HBM and VALU issue (~0.67 of its cycles), so its time on a
    # box whose VALU probe runs below nominal is also quoted scaled to the nominal rate
    if sp or vp:
        box = {k: sp[k] for k in ("stream_copy_GBs", "stream_read_GBs") if k in sp}
        box.update(vp)
        if vp.get("fp64_valu_TFLOPs"):
            box["element_kernel_ms_box_normalized"] = ms_ele * vp["fp64_valu_TFLOPs"] * 1e12 / FP64_VALU_NOMINAL
            box["element_kernel_ms_box_normalized_note"] = ("element kernel ms x (probe fp64 FMA rate / nominal "
                                                            f"{FP64_VALU_NOMINAL / 1e12:g} TFLOP/s)")
        out["box"] = box
    if world == 1:
        tr = pmc_traffic(NE)
        out["roofline"].update(tr)
        if out["roofline"].get("traffic"):
            out["roofline"]["frac_actual"] = out["roofline"]["traffic"] / (ms_ele * 1e-3) / HBM_PEAK
            if sp:   # measured bytes against the measured ceilings (the canonical count exceeds the bytes moved)
                out["roofline"]["frac_of_stream_copy_actual"] = (out["roofline"]["traffic"] / (ms_ele * 1e-3) / 1e9
                                                                 / sp["stream_copy_GBs"])
                # the element kernel reads ~4x what it writes: its fairest ceiling is the box's read-only rate
                out["roofline"]["frac_of_stream_read_actual"] = (out["roofline"]["traffic"] / (ms_ele * 1e-3) / 1e9
                                                                 / sp["stream_read_GBs"])
        rt = tr.get("riv_traffic")
        if rt and ms_riv > 0:
            out["roofline"]["riv_frac_actual"] = rt / (ms_riv * 1e-3) / HBM_PEAK

    # the sections below are side measurements beside the headline value: a failure in one is recorded in the line
    # (and on stderr) instead of discarding the measured value
    def side(key, fn):
        try:
            out[key] = fn()
        except Exception as e:  # noqa: BLE001
            print(f"[bench] {key} failed: {e!r}", file=sys.stderr, flush=True)
            out[key] = {"error": repr(e)}

    hb("side")
    if not args.no_host_vectors and world == 1:
        def host_vectors():
            y_h = np.ascontiguousarray(y_loc)
            dy_h = np.empty_like(y_h)
            h.eval(0.0, y_h, dy_h)
            th = time.perf_counter()
            nrep = 5
            for _ in range(nrep):
                h.eval(0.0, y_h, dy_h, raise_on_physics=False)
            out["host_vector_note"] = ("PCIe-inclusive: y H2D + RHS + ydot D2H + error-word read per eval (the "
                                       "reference f's host N_Vector contract), never `value`")
            return NE * nrep / (time.perf_counter() - th)
        side("host_vector_value", host_vectors)

    def fresh_handle():
        hh = runtime.RhsHandle(gm, mode=mode, device=local, stream=stream.cuda_stream)
        hh.set_step_inputs()
        hh.eval_device(0.0, yp, dyp)
        return hh
    # the integrator first, on the default handle: its ~25 NY-long vectors are then allocated the way a SHUD run
    # allocates them (at startup), not into device memory the many-class handles just fragmented
    if world == 1 and not args.no_ode:
        def integrator():
            h.set_step_inputs()        # the state a fresh handle starts from (step inputs + carried state reset)
            h.eval_device(0.0, yp, dyp)
            return ode_timing(h, y_glob, ms_eval, warm_steps=int(os.environ.get("SHUD_BENCH_ODE_WARM", "0")))
        side("integrator", integrator)
    if world == 1 and not args.no_many_class:
        h.close()                      # free the default handle's device memory first
        h = None
        side("many_class", lambda: many_class_timing(gm, y_glob, mode, local, args.steps, max(3, args.settle)))
    if world == 1 and not args.no_et:
        if h is None:
            h = fresh_handle()
        side("et_prelude", lambda: et_prelude_timing(h, gm))
    if world == 1 and rank == 0 and args.e2e_ele > 0:
        side("end_to_end", lambda: e2e_timing(args.e2e_ele))

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        side("cpu_baseline", lambda: cpu_baseline(gm, y_glob, mode, args.cpu_seconds))
    if world > 1:
        dist.barrier()
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if h is not None:
        h.close()
    hb("report")
    if world > 1:
        dist.destroy_process_group()
    if arm:
        import faulthandler
        faulthandler.cancel_dump_traceback_later()


def parity_vs_1gpu(h, gm, y_glob, part, mode, local, stream, yp, dyp, dy_t, dist, calls=2):
    """After the timed loop: every rank's owned DY, bit for bit, against a full-mesh single-GPU handle evaluated on
    the rank's own device at the same global state.  Both handles restart from the same step inputs and carried
    state (set_step_inputs), then make `calls` successive stateful evaluations; the partitioned ones run the full
    device eval (pack, RCCL exchange, folded launch) collectively across the ranks."""
    import torch
    from shud_rhs import partition, runtime
    h.set_step_inputs()
    full = runtime.RhsHandle(gm, mode=mode, device=local, stream=stream.cuda_stream)
    full.set_step_inputs()
    yg = torch.from_numpy(y_glob).to(f"cuda:{local}")
    dyg = torch.empty_like(yg)
    ok, words = True, 0
    for _ in range(calls):
        h.eval_device(0.0, yp, dyp)
        full.eval_device(0.0, yg.data_ptr(), dyg.data_ptr())
        torch.cuda.synchronize()
        got = dy_t.cpu().numpy()
        want = partition.local_state(dyg.cpu().numpy(), gm, part)
        ok &= bool(np.array_equal(got, want, equal_nan=True))
        words += got.size
    e1, e2 = h.get_error(), full.get_error()
    ok &= not (int(e1["flags"]) & FATAL_FLAGS) and int(e1["flags"]) == int(e2["flags"])
    full.close()
    del yg, dyg
    torch.cuda.empty_cache()
    n_ok = 1 if ok else 0
    if dist is not None:
        t = torch.tensor([n_ok], dtype=torch.int64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        n_ok = int(t.item())
        world = dist.get_world_size()
    else:
        world = 1
    return {"ok": ok, "all_ok": n_ok == world, "ranks_ok": n_ok, "calls": calls, "words_checked_rank0": words,
            "note": "each rank's owned DY after set_step_inputs + 2 stateful device evals (RCCL exchange, folded "
                    "launch) vs a full-mesh single-GPU handle on the same device: np.array_equal (NaN == NaN)"}


def e2e_timing(n_ele, days=1.0):
    """SHUD() end to end through the C++ host (shud-up_amd/shud_gpu): a synthetic project written
    in SHUD text format (seeded mesh + river tree, hourly forcing, 24 hourly outputs), run for `days` simulated
    days as a child process; its own timing line is reported (loop_s = the time loop, wall_s incl. load)."""
    import subprocess
    import tempfile
    from shud_rhs import synth
    exe = os.path.join(ROOT, "shud-up_amd", "shud_gpu")
    with tempfile.TemporaryDirectory() as d:
        synth.write_project(d, "syn", n_ele, days=days)
        r = subprocess.run([exe, "-q", "-o", os.path.join(d, "out"), "-C", d, d, "syn"], capture_output=True,
                           text=True, timeout=300)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith('{"shud_gpu"')]
        if r.returncode != 0 or not line:
            return {"error": f"shud_gpu exit {r.returncode}: {(r.stderr or r.stdout)[-300:]}"}
        res = json.loads(line[-1])["shud_gpu"]
    res["simulated_days_per_s"] = days / res["loop_s"] if res["loop_s"] > 0 else None
    res["note"] = ("shud_gpu (C++ host: readers, forcing/TSR, device ET prelude + RHS + integrator + outputs) on a "
                   f"synthetic {n_ele}-element project, {days:g} simulated day(s), hourly forcing and outputs")
    return res


def ode_timing(h, y0, ms_eval, max_steps=40, budget_s=4.0, warm_steps=0):
    """The device integrator (shud_ode_solve, SURVEY §8f f2: CVODE BDF/Newton/SPGMR as SetCVODE configures it,
    ccw's cfg.para tolerances) on the same mesh and handle: internal steps (CV_ONE_STEP) from the bench state,
    y never leaving HBM.  rhs_share = RHS evaluations x the RHS time measured above / wall time: the rest is
    the fused N_Vector kernels plus the host's scalar control (one small D2H per Newton/Krylov iteration)."""
    from shud_rhs.runtime import OdeSolver
    ode = OdeSolver(h, 0.0, y0, 1e-4, 1e-4, 1e-2, 30.0)
    flag, _, _ = ode.solve(1e9, one_step=True, y_out=False)        # first step: setup outside the timing
    # warm_steps (SHUD_BENCH_ODE_WARM, default 0) more untimed steps: not a clock effect here — 5 of them time steps
    # 7-46 instead of 2-41, where the solver runs order 2 with 128 instead of 117 RHS evaluations and 211 instead of
    # 201 host syncs per 40 steps (4.85 vs 4.39 ms per step on one box, profiles/r05/ode_warm/), so the default keeps
    # the steps every earlier round timed
    for _ in range(warm_steps):
        if flag < 0:
            break
        flag, _, _ = ode.solve(1e9, one_step=True, y_out=False)
    s0 = ode.stats()
    n, t0 = 0, time.perf_counter()
    while flag >= 0 and n < max_steps and time.perf_counter() - t0 < budget_s:
        flag, _, _ = ode.solve(1e9, one_step=True, y_out=False)
        n += 1
    wall = time.perf_counter() - t0
    s1 = ode.stats()
    ode.close()
    d = {k: s1[k] - s0[k] for k in ("nst", "nfe", "nfe_ls", "nni", "nli", "netf", "ncfn", "n_sync")}
    nrhs = d["nfe"] + d["nfe_ls"]
    return {"flag": flag, "steps": d["nst"], "rhs_evals": nrhs, "newton_iters": d["nni"], "krylov_iters": d["nli"],
            "host_syncs": d["n_sync"], "ms_per_step": wall / max(1, d["nst"]) * 1e3,
            "ms_per_rhs_eval_incl_solver": wall / max(1, nrhs) * 1e3,
            "rhs_share": nrhs * ms_eval * 1e-3 / wall if wall > 0 else None,
            "t_reached_min": s1["tcur"], "order": s1["qcur"], "h_min": s1["hcur"],
            "warm_steps": 1 + warm_steps,
            "note": "CV_ONE_STEP internal steps from the bench state (reltol 1e-4, abstol 1e-4, InitStep 1e-2, "
                    "MaxStep 30 min), serial-semantics RHS, state in HBM; the first 1 + warm_steps steps untimed"}


def et_prelude_timing(h, gm, reps=10):
    """The ET-step prelude on the device (shud_et_step) on the same mesh: synthetic statics and
    forcing rows (4 stations, terrain radiation recomputed each step), once per ET step — not per RHS.  Each
    call ends with the error-word read, like the reference's myexit checks."""
    from shud_rhs import abi, et
    etm = et.synth_et(gm.num_ele, seed=4)
    h.et_attach(etm)
    fs = [et.synth_forcing(60.0 * k, 60.0, seed=k, tsr_mode=abi.SHUD_TSR_RECOMPUTE) for k in range(reps + 3)]
    for f in fs[:3]:
        h.et_step(f)
    t0 = time.perf_counter()
    for f in fs[3:]:
        h.et_step(f)
    ms = (time.perf_counter() - t0) / reps * 1e3
    # bytes the kernel moves per element: statics 92 + carried r/w 48 + outputs 16x8 + packed records 40
    b_ele = 92 + 48 + 128 + 40
    return {"ms_per_step": ms, "bytes_per_element": b_ele, "achieved_GBs": b_ele * gm.num_ele / (ms * 1e-3) / 1e9,
            "note": "per ET step (not per RHS); replaces a 56 B/element host->device upload of step inputs "
                    "plus the host's tReadForcing/ET loops"}


def stream_probe(dev, n=1 << 27, reps=20):
    """STREAM probes (shud-up_amd/libshud_stream.so; configurations from tools/stream_sweep.hip), 1 GiB buffers, HIP-event timed on torch's current stream:
    the best of three copy kernels (bytes read + written) and a read-only sweep (bytes read): the practical
    HBM ceilings of this box for a copy and for a read-dominated stream."""
    import ctypes
    import torch
    lib = ctypes.CDLL(os.path.join(ROOT, "shud-up_amd", "libshud_stream.so"))
    lib.shud_stream_copy_v.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_int]
    a = torch.ones(n, dtype=torch.float64, device=f"cuda:{dev}")
    b = torch.empty_like(a)
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for v in (0, 1, 2, 3):
        for _ in range(3):
            lib.shud_stream_copy_v(a.data_ptr(), b.data_ptr(), 8 * n, st, v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            lib.shud_stream_copy_v(a.data_ptr(), b.data_ptr(), 8 * n, st, v)
        e1.record()
        torch.cuda.synchronize()
        sec = e0.elapsed_time(e1) * 1e-3
        if v < 3:
            ok = bool(torch.equal(a[:4096], b[:4096])) and bool(torch.equal(a[-4096:], b[-4096:]))
            res[v] = 2 * 8 * n * reps / sec / 1e9 if ok else None
            b.zero_()
        else:
            res[v] = 8 * n * reps / sec / 1e9
    del a, b
    torch.cuda.empty_cache()
    names = {0: "grid-stride nt", 1: "one-shot x4 nt-load nt-store", 2: "one-shot x1 nt-store"}
    best = max((k for k in (0, 1, 2) if res[k]), key=lambda k: res[k], default=None)
    if best is None:
        return {}
    return {"stream_copy_GBs": res[best], "stream_copy_kernel": names[best],
            "stream_copy_all_GBs": {names[k]: res[k] for k in (0, 1, 2)}, "stream_read_GBs": res[3]}


def valu_probe(dev, blocks=2048, iters=4000, reps=5):
    """fp64 VALU probe (shud-up_amd/libshud_stream.so shud_valu_probe): 8 independent fma chains per lane, 8 waves per
    SIMD, non-trivial operands, HIP-event timed on torch's current stream, best of `reps` launches after 3 warm-ups;
    and the in-kernel clock = s_memtime / s_memrealtime x 100 MHz stamped by every workgroup (median)."""
    import ctypes
    import torch
    lib = ctypes.CDLL(os.path.join(ROOT, "shud-up_amd", "libshud_stream.so"))
    lib.shud_valu_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(256, dtype=torch.float64, device=f"cuda:{dev}")
    stamps = torch.zeros(2 * blocks, dtype=torch.int64, device=f"cuda:{dev}")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        if lib.shud_valu_probe(blocks, iters, sink.data_ptr(), stamps.data_ptr(), st) != 0:
            return {}
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.shud_valu_probe(blocks, iters, sink.data_ptr(), stamps.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        sec = e0.elapsed_time(e1) * 1e-3
        best = sec if best is None else min(best, sec)
    st_h = stamps.cpu().numpy().reshape(-1, 2).astype(np.float64)
    ok = st_h[:, 1] > 0
    clock = float(np.median(st_h[ok, 0] / st_h[ok, 1])) * 0.1 if ok.any() else None     # GHz (100 MHz ticks)
    flops = 2.0 * blocks * 256 * iters * 128
    rate = flops / best
    del sink, stamps
    return {"fp64_valu_TFLOPs": rate / 1e12, "fp64_valu_frac_nominal": rate / FP64_VALU_NOMINAL,
            "clock_GHz_in_kernel": clock, "valu_probe_ms": best * 1e3,
            "valu_probe_note": "fp64 FMA chains, 8 waves/SIMD, best of 5 launches; clock = s_memtime / s_memrealtime"}


def kernel_src_hash():
    """sha256 (16 hex) over the sources the RHS kernels are built from: keys profiles/pmc_summary.json so a
    PMC traffic figure is only reported for the kernel build it was measured on."""
    import hashlib
    hh = hashlib.sha256()
    csrc = os.path.join(ROOT, "shud-up_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.startswith(("shud_ele_packed", "shud_kernels", "shud_dev", "shud_physics", "shud_rhs.cpp",
                         "shud_handle", "shud_pow")):
            with open(os.path.join(csrc, f), "rb") as fh:
                hh.update(f.encode() + b"\0" + fh.read())
    with open(os.path.join(ROOT, "shud-up_amd", "Makefile"), "rb") as fh:
        hh.update(fh.read())
    return hh.hexdigest()[:16]


def pmc_traffic(NE, kname="shud_ele_kernel"):
    """roofline.traffic from profiles/pmc_summary.json (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, gfx950
    correction, tools/pmc_summary.py) when it was measured on this mesh AND this kernel build; else null."""
    pmc = os.path.join(ROOT, "profiles", "pmc_summary.json")
    src = kernel_src_hash()
    out = {"traffic": None, "kernel_src_hash": src}
    if not os.path.exists(pmc):
        out["traffic_note"] = "no PMC summary"
        return out
    try:
        with open(pmc) as f:
            pj = json.load(f)
    except Exception as e:  # noqa: BLE001
        out["traffic_note"] = f"unreadable PMC summary: {e}"
        return out
    if pj.get("num_ele") != NE or pj.get("kernel_src_hash") != src:
        out["traffic_note"] = (f"PMC summary is stale (measured on num_ele {pj.get('num_ele')}, kernel build "
                               f"{pj.get('kernel_src_hash')}): traffic not reported")
        return out
    k = pj.get("kernels", {})
    if kname in k:
        out["traffic"] = k[kname]["hbm_bytes_per_launch"]
        out["traffic_source"] = ("profiles/pmc_summary.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE; per-pattern "
                                 "gfx950 calibration, profiles/r03/pmc_calib/)")
        if "hbm_bytes_blanket_x2" in k[kname]:
            out["traffic_blanket_x2"] = k[kname]["hbm_bytes_blanket_x2"]
    if "shud_riv_kernel" in k:
        out["riv_traffic"] = k["shud_riv_kernel"]["hbm_bytes_per_launch"]
        if "hbm_bytes_blanket_x2" in k["shud_riv_kernel"]:
            out["riv_traffic_blanket_x2"] = k["shud_riv_kernel"]["hbm_bytes_blanket_x2"]
    return out


def many_class_timing(gm, y, mode, dev, steps, warm=200):
    """The same syn-10M mesh with per-element calibrated parameters: KsatH perturbed by (1 + 1e-7 k), k =
    element mod 400, so the distinct parameter tuples (classes) grow from 33 to 13,200 — more than the 128 one
    workgroup's LDS copy of the class table holds.  "auto": the layout the handle picks (the hybrid layout: KsatH
    streamed per element, 33 classes in LDS); "l2_class_table": the packed layout with its class table read from L2
    (SHUD_RHS_HYB=0, SHUD_RHS_L2_CLASS=1); "soa": the SoA kernel (SHUD_RHS_HYB=0).  Timed like the headline
    (device-resident y, K evals)."""
    import copy
    import torch
    from shud_rhs import runtime
    res = {}
    base = gm.par["KsatH"]
    y_t = torch.from_numpy(y).to(f"cuda:{dev}")
    dy_t = torch.empty_like(y_t)
    m2 = copy.copy(gm)
    m2.par = dict(gm.par)
    m2.par["KsatH"] = base * (1.0 + 1e-7 * (np.arange(gm.num_ele) % 400))
    for name, env in (("auto", {}), ("l2_class_table", {"SHUD_RHS_HYB": "0", "SHUD_RHS_L2_CLASS": "1"}),
                      ("soa", {"SHUD_RHS_HYB": "0"})):
        os.environ.update(env)
        try:
            h = runtime.RhsHandle(m2, mode=mode, device=dev, stream=torch.cuda.current_stream().cuda_stream)
        finally:
            for k in env:
                os.environ.pop(k, None)
        h.set_step_inputs()
        lay = h.layout()
        # untimed evals first, as many as the headline's clock settle: a fresh handle's first evals follow seconds of
        # host-side setup with the GPU idle and run inside the clock ramp (3 evals: element kernel 0.659-0.679 ms;
        # 60: 0.581-0.586 ms on the same box, profiles/r05/mc_warm/)
        for _ in range(warm):
            h.eval_device(0.0, y_t.data_ptr(), dy_t.data_ptr())
        h.timing(steps, 5 if steps >= 20 else 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            h.eval_device(0.0, y_t.data_ptr(), dy_t.data_ptr())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        me, mr, mv, n = h.timing_read()
        h.close()
        res[name] = {"layout": ("hybrid" if lay.get("streamed_fields") else "packed") if lay["packed"] else "soa",
                     "n_classes": 13200 if not lay["packed"] else lay["n_classes"],
                     "streamed_fields": lay.get("streamed_fields", 0), "value": gm.num_ele * steps / dt,
                     "ms_per_step": dt / steps * 1e3, "ele_kernel_ms": me, "riv_kernel_ms": mr}
    torch.cuda.empty_cache()
    return res


def cpu_baseline(gm, y, mode, budget_s):
    """The CPU restatement (oracle/, C + OpenMP, reference loop structure) on this host's cores, on the same
    10M mesh and state: a bounded number of RHS calls (~budget_s of CPU work)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    oracle.set_threads(threads)
    o = oracle.OracleRhs(gm, mode)
    o.set_step_inputs()
    o.eval(0.0, y)                          # warm-up (first-touch)
    n, t0 = 0, time.perf_counter()
    while True:
        o.eval(0.0, y)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 40:
            break
    out = {"value": gm.num_ele * n / el, "unit": "element-flux-updates/s", "cores": threads, "kind": "port",
           "sample": f"{n} RHS calls of the CPU restatement (oracle/shud_oracle.c, OpenMP {threads} threads) on "
                     f"the full syn-10M mesh, {el:.1f}s wall"}
    # the same restatement on 1 thread (SURVEY §8d asks for both), a bounded sample of ~budget_s / 3
    oracle.set_threads(1)
    n1, t1 = 0, time.perf_counter()
    while True:
        o.eval(0.0, y)
        n1 += 1
        el1 = time.perf_counter() - t1
        if el1 >= budget_s / 3 or n1 >= 10:
            break
    out["value_1thread"] = gm.num_ele * n1 / el1
    out["sample_1thread"] = f"{n1} RHS calls on 1 thread, {el1:.1f}s wall"
    oracle.set_threads(threads)
    return out


if __name__ == "__main__":
    main()
