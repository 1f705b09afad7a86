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
def test_k_rank_simulation_bit_identical(nranks, mode):
    import oracle
    m, y = cases.variant(6000, seed=21)
    g = oracle.OracleRhs(m, mode)
    g.set_step_inputs()
    _, _, plans = partition.build_plans(m, nranks)
    locs = [partition.local_model(m, plans[r], r, nranks) for r in range(nranks)]
    parts = [p for _, p in locs]
    ors = []
    for lm, part in locs:
        o = oracle.OracleRhs(lm, mode)
        o.set_step_inputs()
        ors.append(o)
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
                dy_ext = ors[r].eval(0.0, partition.extended_state(owned[r], gele, griv, part))[0]
                got = partition.owned_dy(dy_ext, lm, part)
                want = partition.local_state(ref, m, part)
                assert np.array_equal(got, want), f"rank {r} call {call}"


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
    m, y = cases.variant(5000, seed=44)
    _, _, plans = partition.build_plans(m, world)
    lm, part = partition.local_model(m, plans[rank], rank, world)
    o = oracle.OracleRhs(lm, 0)
    o.set_step_inputs()
    ok = True
    for call in range(3):
        owned = partition.local_state(y, m, part)
        eb, rb = partition.pack_send(owned, part)
        gele = np.zeros(3 * (part.ele_gid.size - part.n_own_ele))
        griv = np.zeros(part.riv_gid.size - part.n_own_riv)
        reqs = []
        for p in range(world):
            if p == rank:
                continue
            s0, s1 = part.ele_send_off[p], part.ele_send_off[p + 1]
            r0, r1 = part.ele_recv_off[p], part.ele_recv_off[p + 1]
            sbuf = torch.from_numpy(np.ascontiguousarray(eb[3 * s0:3 * s1]))
            rbuf = torch.zeros(3 * (r1 - r0), dtype=torch.float64)
            rs0, rs1 = part.riv_send_off[p], part.riv_send_off[p + 1]
            rr0, rr1 = part.riv_recv_off[p], part.riv_recv_off[p + 1]
            sriv = torch.from_numpy(np.ascontiguousarray(rb[rs0:rs1]))
            rriv = torch.zeros(rr1 - rr0, dtype=torch.float64)
            reqs += [dist.isend(sbuf, p), dist.irecv(rbuf, p), dist.isend(sriv, p, tag=1), dist.irecv(rriv, p, tag=1)]
            for q in reqs:
                q.wait()
            gele[3 * r0:3 * r1] = rbuf.numpy()
            griv[rr0:rr1] = rriv.numpy()
        dy = partition.owned_dy(o.eval(0.0, partition.extended_state(owned, gele, griv, part))[0], lm, part)
        g = oracle.OracleRhs(m, 0)
        g.set_step_inputs()
        for _ in range(call + 1):
            ref = g.eval(0.0, y)[0]
        ok &= bool(np.array_equal(dy, partition.local_state(ref, m, part)))
    with open(os.path.join(outdir, f"rank{rank}.txt"), "w") as f:
        f.write("ok" if ok else "fail")
    dist.destroy_process_group()


def test_gloo_world_size_2(tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_gloo_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        assert (tmp_path / f"rank{r}.txt").read_text() == "ok"
