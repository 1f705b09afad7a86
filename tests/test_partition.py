"""CPU: mesh partition + halo plans.  Each rank evaluates its local (owned + ghost) mesh with
the CPU oracle after receiving ghost states through the same plan the GPU handle uses; its owned DY must
equal the unpartitioned result bit for bit.  (1) in-process k-rank simulation, (2) world_size-2 gloo run
over torch.distributed (127.0.0.1)."""
import os
import socket

import numpy as np
import pytest

import cases
from shud_rhs import partition, workload


def _global_reach_order(lm, part):
    """The oracle sums a junction's upstream reaches in ascending LOCAL reach order; the GPU handle orders them
    by global id (ShudPartition.riv_gid), as the reference's single loop does (MD_f.cpp:236-240).  Local reach
    order is [owned | ghosts by source rank], so give the oracle a copy of the local model whose reaches are
    re-sorted by global id; returns (model, to_oracle(y_ext), from_oracle(dy_ext))."""
    import copy
    perm = np.argsort(part.riv_gid, kind="stable")          # oracle reach k = local reach perm[k]
    inv = np.empty_like(perm)
    inv[perm] = np.arange(perm.size)
    lo = copy.copy(lm)
    lo.riv = {k: v[perm] for k, v in lm.riv.items()}
    d = lm.riv_down[perm]
    lo.riv_down = np.where(d >= 0, inv[np.where(d >= 0, d, 0)], d).astype(np.int32)
    lo.riv_bc = lm.riv_bc[perm]
    lo.seg_riv = inv[lm.seg_riv].astype(np.int32)
    NE3 = 3 * lm.num_ele

    def to_o(y):
        return np.concatenate([y[:NE3], y[NE3:NE3 + perm.size][perm]])

    def from_o(dy):
        out = dy.copy()
        out[NE3 + perm] = dy[NE3:NE3 + perm.size]
        return out
    return lo.finalize(), to_o, from_o


def _ghost_from_peers(parts, packs, r):
    """Assemble rank r's ghost buffers from every peer's packed send buffers (the all-to-all-v)."""
    P = len(parts)
    pr = parts[r]
    gele = np.zeros(3 * (pr.ele_gid.size - pr.n_own_ele))
    griv = np.zeros(pr.riv_gid.size - pr.n_own_riv)
    for p in range(P):
        if p == r:
            continue
        eb, rb = packs[p]
        s0, s1 = parts[p].ele_send_off[r], parts[p].ele_send_off[r + 1]
        d0, d1 = pr.ele_recv_off[p], pr.ele_recv_off[p + 1]
        assert s1 - s0 == d1 - d0
        gele[3 * d0:3 * d1] = eb[3 * s0:3 * s1]
        s0, s1 = parts[p].riv_send_off[r], parts[p].riv_send_off[r + 1]
        d0, d1 = pr.riv_recv_off[p], pr.riv_recv_off[p + 1]
        assert s1 - s0 == d1 - d0
        griv[d0:d1] = rb[s0:s1]
    return gele, griv


@pytest.mark.parametrize("nranks", [2, 3, 4])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("planner", ["python", "cpp"])
def test_k_rank_simulation_bit_identical(nranks, mode, planner):
    import oracle
    m, y = cases.variant(6000, seed=21)
    g = oracle.OracleRhs(m, mode)
    g.set_step_inputs()
    if planner == "python":
        _, _, plans = partition.build_plans(m, nranks)
        locs = [partition.local_model(m, plans[r], r, nranks) for r in range(nranks)]
    else:
        ep, _ = partition.cpp_partition(m, nranks, partition.PART_MULTILEVEL)
        locs = [partition.CppPlan(m, ep, nranks, r).local_model() for r in range(nranks)]
    parts = [p for _, p in locs]
    ors = []
    for lm, part in locs:
        lo, to_o, from_o = _global_reach_order(lm, part)
        o = oracle.OracleRhs(lo, mode)
        o.set_step_inputs()
        ors.append((o, to_o, from_o))
    assert sum(p.n_own_ele for p in parts) == m.num_ele
    assert sum(p.n_own_riv for p in parts) == m.num_riv
    ys = [y, workload.random_state(m, seed=5)]
    for yy in ys:
        for call in range(2):
            ref = g.eval(0.0, yy)[0]
            owned = [partition.local_state(yy, m, p) for p in parts]
            packs = [partition.pack_send(owned[r], parts[r]) for r in range(nranks)]
            for r, (lm, part) in enumerate(locs):
                gele, griv = _ghost_from_peers(parts, packs, r)
                ge_ref, gr_ref = partition.ghost_values(yy, m, part)
                assert np.array_equal(gele, ge_ref) and np.array_equal(griv, gr_ref)
                o, to_o, from_o = ors[r]
                dy_ext = from_o(o.eval(0.0, to_o(partition.extended_state(owned[r], gele, griv, part)))[0])
                got = partition.owned_dy(dy_ext, lm, part)
                want = partition.local_state(ref, m, part)
                assert np.array_equal(got, want, equal_nan=True), f"rank {r} call {call}"


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_interior_prefix(nranks):
    """Owned elements are numbered [interior | boundary]: the interior prefix reads no ghost data (the GPU
    handle runs it while the halo exchange is in flight) and it is most of the owned set."""
    m, _ = cases.variant(20000, seed=5)
    _, _, plans = partition.build_plans(m, nranks)
    for r in range(nranks):
        lm, part = partition.local_model(m, plans[r], r, nranks)
        own = part.n_own_ele
        nab = lm.nabr.reshape(3, -1)[:, :own]
        dep = (nab >= own).any(0)
        bad = np.zeros(lm.num_ele, bool)
        np.logical_or.at(bad, lm.seg_ele[lm.seg_riv >= part.n_own_riv], True)
        dep |= bad[:own]
        n_int = int(np.argmax(dep)) if dep.any() else own
        assert not dep[:n_int].any() and dep[n_int:].all(), "owned elements not ordered [interior | boundary]"
        assert n_int >= 0.8 * own


def test_edge_cut_counts():
    m, _ = cases.variant(20000, seed=5)
    one = np.zeros(m.num_ele, dtype=np.int32)
    assert partition.edge_cut(m, one) == (0, 0)
    ep, _, _ = partition.build_plans(m, 4)
    ce, cs = partition.edge_cut(m, ep)
    nab = m.nabr.reshape(3, -1)
    brute = sum(1 for j in range(3) for i in range(m.num_ele)
                if nab[j, i] > i and ep[i] != ep[nab[j, i]])
    assert ce == brute and 0 < ce < 0.1 * m.num_ele and cs >= 0


def test_rcb_balance():
    m = cases.variant(20000, seed=3)[0]
    ep, rp = partition.assign_owners(m, 8)
    w = 1.0 + np.bincount(m.seg_ele, minlength=m.num_ele)
    loads = np.bincount(ep, weights=w, minlength=8)
    assert loads.max() / loads.mean() < 1.05


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(os.path.dirname(here), "shud-up_amd"), os.path.join(os.path.dirname(here), "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(here))
    import bench
    m, y = cases.variant(5000, seed=44)
    # bench.py's N > 1 partition: rank 0 partitions, the map and stats are broadcast (here over gloo)
    ep, pst = bench.shared_partition(m, world, rank, dist, "cpu")
    ref, rst = partition.cpp_partition(m, world, partition.PART_AUTO, seed=12345)
    same = {k: v for k, v in pst.items() if k != "seconds"} == {k: v for k, v in rst.items() if k != "seconds"}
    if not (np.array_equal(ep, ref) and same):
        with open(os.path.join(outdir, f"rank{rank}.txt"), "w") as f:
            f.write("fail: broadcast partition differs")
        dist.destroy_process_group()
        return
    lm, part = partition.CppPlan(m, ep, world, rank).local_model()
    lo, to_o, from_o = _global_reach_order(lm, part)
    o = oracle.OracleRhs(lo, 0)
    o.set_step_inputs()
    ok = True
    for call in range(3):
        owned = partition.local_state(y, m, part)
        eb, rb = partition.pack_send(owned, part)
        gele = np.zeros(3 * (part.ele_gid.size - part.n_own_ele))
        griv = np.zeros(part.riv_gid.size - part.n_own_riv)
        reqs, recv = [], []
        for p in range(world):            # post every send / receive first, then wait: no pairwise ordering
            if p == rank:
                continue
            s0, s1 = part.ele_send_off[p], part.ele_send_off[p + 1]
            r0, r1 = part.ele_recv_off[p], part.ele_recv_off[p + 1]
            rs0, rs1 = part.riv_send_off[p], part.riv_send_off[p + 1]
            rr0, rr1 = part.riv_recv_off[p], part.riv_recv_off[p + 1]
            # empty messages are skipped on both sides (the peer's counts mirror these)
            if s1 > s0:
                reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(eb[3 * s0:3 * s1])), p, tag=0))
            if rs1 > rs0:
                reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(rb[rs0:rs1])), p, tag=1))
            if r1 > r0:
                t = torch.zeros(3 * (r1 - r0), dtype=torch.float64)
                reqs.append(dist.irecv(t, p, tag=0))
                recv.append((gele, 3 * r0, t))
            if rr1 > rr0:
                t = torch.zeros(rr1 - rr0, dtype=torch.float64)
                reqs.append(dist.irecv(t, p, tag=1))
                recv.append((griv, rr0, t))
        for q in reqs:
            q.wait()
        for buf, off, t in recv:
            buf[off:off + t.numel()] = t.numpy()
        dy_ext = from_o(o.eval(0.0, to_o(partition.extended_state(owned, gele, griv, part)))[0])
        dy = partition.owned_dy(dy_ext, lm, part)
        g = oracle.OracleRhs(m, 0)
        g.set_step_inputs()
        for _ in range(call + 1):
            ref = g.eval(0.0, y)[0]
        ok &= bool(np.array_equal(dy, partition.local_state(ref, m, part)))
    with open(os.path.join(outdir, f"rank{rank}.txt"), "w") as f:
        f.write("ok" if ok else "fail")
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_world_size(tmp_path, world):
    """world_size 2 and 4 over gloo (127.0.0.1): rank 0 builds the C++ partition and broadcasts it (bench.py's
    shared_partition), each rank builds its own C++ plan, trades halos point to point, evaluates its local mesh
    with the oracle: owned DY bit-identical."""
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_gloo_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        assert (tmp_path / f"rank{r}.txt").read_text() == "ok"


# ---------------------------------------------------------------------------------------------------------
# the C++ partitioner / planner (include/shud_partition.h) against the Python restatement above
# ---------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("nparts", [1, 2, 3, 4, 8])
def test_cpp_rcb_matches_python(nparts):
    m = cases.variant(20000, seed=3)[0]
    ep_py, _ = partition.assign_owners(m, nparts)
    ep, st = partition.cpp_partition(m, nparts, partition.PART_RCB)
    assert np.array_equal(ep, ep_py)
    assert (st["edge_cut"], st["segment_cut"]) == partition.edge_cut(m, ep)


@pytest.mark.parametrize("nparts", [2, 4, 8])
@pytest.mark.parametrize("method", [partition.PART_MULTILEVEL, partition.PART_RCB])
def test_cpp_plans_match_python(nparts, method):
    """Given the same element partition, the C++ plan and local mesh equal the Python ones array for array."""
    m = cases.variant(20000, seed=5)[0]
    m.step = workload.random_step_inputs(m, seed=3)
    ep, _ = partition.cpp_partition(m, nparts, method)
    ep_py, rp_py, plans = partition.build_plans(m, nparts, ele_part=ep)
    ge, gr = partition.cpp_halo(m, ep)
    for r in range(nparts):
        pl = partition.CppPlan(m, ep, nparts, r)
        assert np.array_equal(pl.riv_part, rp_py)
        lm_py, pa = partition.local_model(m, plans[r], r, nparts)
        lm, pc = pl.local_model()
        for k in ["ele_gid", "riv_gid", "seg_gid", "ele_send_off", "ele_send_idx", "ele_recv_off", "riv_send_off",
                  "riv_send_idx", "riv_recv_off"]:
            assert np.array_equal(np.asarray(getattr(pa, k)), np.asarray(getattr(pc, k))), f"rank {r} {k}"
        assert (pa.n_own_ele, pa.n_own_riv) == (pc.n_own_ele, pc.n_own_riv)
        for d_py, d_c in ((lm_py.ele, lm.ele), (lm_py.riv, lm.riv), (lm_py.par, lm.par), (lm_py.step, lm.step)):
            assert set(d_py) == set(d_c)
            for k in d_py:
                assert np.array_equal(d_py[k], d_c[k]), k
        for k in ["nabr", "ibc", "iss", "riv_down", "riv_bc", "seg_ele", "seg_riv", "seg_length", "seg_cwr"]:
            assert np.array_equal(getattr(lm_py, k), getattr(lm, k)), k
        y = workload.random_state(m, seed=r)
        assert np.array_equal(pl.owned_state(y), partition.local_state(y, m, pc))
        assert ge[r] == pl.ele_gid.size - pl.n_own_ele and gr[r] == pl.riv_gid.size - pl.n_own_riv
        pl.close()


@pytest.mark.parametrize("name", ["ccw", "heihe"])
@pytest.mark.parametrize("nparts", [2, 4, 8])
def test_multilevel_partition_properties(name, nparts):
    """Multilevel partitions of the reference's basin meshes: deterministic per seed, every part non-empty,
    vertex-weight imbalance within the 1.03 target (plus coarse-vertex slack on these small meshes)."""
    m = getattr(cases, name)()[0]
    ep, st = partition.cpp_partition(m, nparts, partition.PART_MULTILEVEL, seed=7)
    ep2, _ = partition.cpp_partition(m, nparts, partition.PART_MULTILEVEL, seed=7)
    assert np.array_equal(ep, ep2)
    assert np.bincount(ep, minlength=nparts).min() > 0
    w = 1.0 + np.bincount(m.seg_ele, minlength=m.num_ele)
    loads = np.bincount(ep, weights=w, minlength=nparts)
    assert abs(loads.max() / loads.mean() - st["imbalance"]) < 1e-9
    assert st["imbalance"] < 1.04
    assert (st["edge_cut"], st["segment_cut"]) == partition.cpp_edge_cut(m, ep) == partition.edge_cut(m, ep)


def test_multilevel_beats_rcb_on_bisection():
    """Regression guard on partition quality: the 2-way multilevel cut of the 20k jittered-grid mesh is below
    the straight RCB cut in mesh edges and in river segments (measured 76 / 12 vs 108 / 108)."""
    m = cases.variant(20000, seed=17)[0]
    _, ml = partition.cpp_partition(m, 2, partition.PART_MULTILEVEL)
    _, rcb = partition.cpp_partition(m, 2, partition.PART_RCB)
    assert ml["edge_cut"] < rcb["edge_cut"] and ml["segment_cut"] < rcb["segment_cut"]


@pytest.mark.parametrize("case", ["qhh", "qhh_variant"])
@pytest.mark.parametrize("nparts", [2, 3, 4, 8])
def test_lake_plans(case, nparts):
    """Lakes in C++ plans: every lake group (lake elements + bank elements) on one part, each lake owned by
    exactly one rank with its inflowing reaches local there, owned-state round trip with lake stages, local
    lake numbering, balance kept around the locked groups."""
    m, y = getattr(cases, case)()
    ep, st = partition.cpp_partition(m, nparts, partition.PART_MULTILEVEL)
    nab = m.nabr.reshape(3, -1)
    lk = np.nonzero(m.ilake > 0)[0]
    for j in range(3):
        nb = nab[j, lk]
        assert np.all(ep[nb[nb >= 0]] == ep[lk[nb >= 0]])
    assert st["imbalance"] < 1.06
    plans = [partition.CppPlan(m, ep, nparts, r) for r in range(nparts)]
    assert np.array_equal(np.sort(np.concatenate([p.lake_gid for p in plans])), np.arange(m.num_lake))
    y2 = np.zeros_like(y)
    for p in plans:
        o = p.owned_state(y)
        assert o.size == 3 * p.n_own_ele + p.n_own_riv + p.lake_gid.size
        partition._host().shud_plan_scatter_owned(p.h, o.ctypes.data, m.num_ele, y2.ctypes.data)
    assert np.array_equal(y, y2)
    for r, p in enumerate(plans):
        lm, part = p.local_model()
        assert lm.num_lake == part.n_own_lake == p.lake_gid.size
        li = lm.ilake
        assert np.all((li >= 0) & (li <= lm.num_lake))
        assert np.all(np.nonzero(li > 0)[0] < part.n_own_ele)          # lake elements are owned
        for k, gl in enumerate(p.lake_gid):                             # inflowing reaches are local
            inflow = np.nonzero(m.riv_down == -3 - (gl + 1))[0]
            assert np.isin(inflow, p.riv_gid).all()
            loc = np.nonzero(np.isin(p.riv_gid, inflow))[0]
            assert np.all(lm.riv_down[loc] == -3 - (k + 1))
        others = np.nonzero((m.riv_down <= -4) & ~np.isin(-3 - m.riv_down - 1, p.lake_gid))[0]
        assert np.all(lm.riv_down[np.isin(p.riv_gid, others)] == -3)  # into a lake owned elsewhere: outlet code
        p.close()


def test_lake_partition_constraint():
    m, _ = cases.qhh_variant()
    rng = np.random.default_rng(5)
    ep = rng.integers(0, 4, m.num_ele).astype(np.int32)
    with pytest.raises(RuntimeError, match="lake"):
        partition.CppPlan(m, ep, 4, 0)
    ec = partition.cpp_constrain(m, ep, 4)
    assert np.array_equal(partition.cpp_constrain(m, ec, 4), ec)            # idempotent
    moved = np.nonzero(ec != ep)[0]
    assert np.all((m.ilake[moved] > 0) | np.isin(moved, m.nabr.reshape(3, -1)[:, m.ilake > 0]))
    for r in range(4):
        partition.CppPlan(m, ec, 4, r).close()
    m2, _ = cases.variant(3000, seed=4)                                     # no lakes: untouched
    ep2 = rng.integers(0, 3, m2.num_ele).astype(np.int32)
    assert np.array_equal(partition.cpp_constrain(m2, ep2, 3), ep2)
