"""CPU: randomized property tests (hypothesis).  Meshes, states, step inputs, partitions and seeds are
drawn at random; each property is one the reference's algorithm guarantees or one the design promises:

  * the C restatement and the independent numpy restatement agree bit for bit (serial and OMP, stateful calls),
  * interior lateral fluxes are exactly antisymmetric (MD_ElementFlux.cpp:54-80, 122-138, fu_Sub = 1),
  * segment / junction exchange conserves volume (PassValue, MD_f.cpp:217-257),
  * the thread count of the OpenMP oracle does not change a bit (reference reductions are index-ordered),
  * any element partition gives plans that own every element / reach exactly once, whose send and receive
    counts mirror each other, whose C++ and Python forms are identical, and whose k-rank simulation reproduces
    the unpartitioned DY bit for bit,
  * the multilevel partitioner is deterministic per seed, keeps every part non-empty and stays within its
    balance target.
Sizes are small so the whole file runs in well under a minute."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import cases
from shud_rhs import abi, partition, workload

SETTINGS = settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow],
                    derandomize=True)


def _model(n, seed, open_boundary):
    m, y = cases.variant(n, seed=seed)
    m.close_boundary = 0 if open_boundary else 1
    return m, y


@SETTINGS
@given(n=st.integers(300, 3000), seed=st.integers(0, 10_000), mode=st.sampled_from([0, 1]),
       open_boundary=st.booleans(), calls=st.integers(1, 3))
def test_restatements_agree_on_random_meshes(n, seed, mode, open_boundary, calls):
    import numpy_oracle
    import oracle
    m, y = _model(n, seed, open_boundary)
    o, p = oracle.OracleRhs(m, mode), numpy_oracle.NumpyRhs(m, mode)
    o.set_step_inputs()
    p.set_step_inputs()
    for yy in (y, workload.random_state(m, seed=seed + 1)):
        for _ in range(calls):
            a, code, _, _ = o.eval(0.0, yy)
            b = p.eval(0.0, yy)
            assert code == 0
            assert np.all((a == b) | (np.isnan(a) & np.isnan(b)))


@SETTINGS
@given(n=st.integers(300, 3000), seed=st.integers(0, 10_000))
def test_lateral_antisymmetry_and_exchange_conservation(n, seed):
    import oracle
    m, _ = cases.variant(n, seed=seed)
    m.step["fu_sub"] = np.ones(m.num_ele)
    o = oracle.OracleRhs(m, 0)
    o.set_step_inputs()
    o.eval(0.0, workload.random_state(m, seed=seed + 3))
    d = o.diagnostics()
    NE = m.num_ele
    nab = m.nabr.reshape(3, NE)
    qs, qg = d["qele_surf"].reshape(3, NE), d["qele_sub"].reshape(3, NE)
    for j in range(3):
        for i in np.nonzero(nab[j] >= 0)[0]:
            k = nab[j, i]
            back = np.nonzero(nab[:, k] == i)[0]
            if back.size:
                assert qs[j, i] == -qs[back[0], k] and qg[j, i] == -qg[back[0], k]
    tot = np.abs(d["qseg_surf"]).sum() + np.abs(d["qseg_sub"]).sum() + 1e-300
    assert abs(d["qe2r_surf"].sum() + d["qriv_surf"].sum()) <= 1e-12 * tot
    assert abs(d["qe2r_sub"].sum() + d["qriv_sub"].sum()) <= 1e-12 * tot


@SETTINGS
@given(seed=st.integers(0, 10_000), threads=st.sampled_from([1, 2, 3, 5, 8]), mode=st.sampled_from([0, 1]))
def test_oracle_thread_count_invariance(seed, threads, mode):
    import oracle
    m, y = cases.variant(2500, seed=seed)
    oracle.set_threads(1)
    a = oracle.OracleRhs(m, mode)
    a.set_step_inputs()
    ref = a.eval(0.0, y)[0]
    oracle.set_threads(threads)
    b = oracle.OracleRhs(m, mode)
    b.set_step_inputs()
    got = b.eval(0.0, y)[0]
    oracle.set_threads(8)
    assert np.array_equal(ref, got)


@SETTINGS
@given(n=st.integers(400, 4000), seed=st.integers(0, 10_000), nparts=st.integers(2, 6),
       method=st.sampled_from([partition.PART_MULTILEVEL, partition.PART_RCB, -1]))
def test_random_partitions_give_consistent_plans(n, seed, nparts, method):
    """method -1: a random element assignment (worst case for the planner: ragged, disconnected parts)."""
    m, _ = cases.variant(n, seed=seed)
    if method < 0:
        rng = np.random.default_rng(seed)
        ep = rng.integers(0, nparts, m.num_ele).astype(np.int32)
        ep[:nparts] = np.arange(nparts)                 # every part non-empty
    else:
        ep, _ = partition.cpp_partition(m, nparts, method, seed=seed)
    _, rp, plans = partition.build_plans(m, nparts, ele_part=ep)
    parts = [partition.CppPlan(m, ep, nparts, r) for r in range(nparts)]
    own_e = np.concatenate([p.ele_gid[:p.n_own_ele] for p in parts])
    own_r = np.concatenate([p.riv_gid[:p.n_own_riv] for p in parts])
    assert np.array_equal(np.sort(own_e), np.arange(m.num_ele))
    assert np.array_equal(np.sort(own_r), np.arange(m.num_riv))
    for r, p in enumerate(parts):
        assert np.array_equal(p.ele_gid, np.concatenate([plans[r]["own_e"], plans[r]["ghost_e"]]))
        assert np.array_equal(p.riv_gid, np.concatenate([plans[r]["own_r"], plans[r]["ghost_r"]]))
        for q in range(nparts):
            if q == r:
                continue
            # what r sends q == what q expects from r, entity by entity
            s0, s1 = p.ele_send_off[q], p.ele_send_off[q + 1]
            d0, d1 = parts[q].ele_recv_off[r], parts[q].ele_recv_off[r + 1]
            assert s1 - s0 == d1 - d0
            sent = p.ele_gid[p.ele_send_idx[s0:s1]]
            recv = parts[q].ele_gid[parts[q].n_own_ele + d0:parts[q].n_own_ele + d1]
            assert np.array_equal(sent, recv)
            s0, s1 = p.riv_send_off[q], p.riv_send_off[q + 1]
            d0, d1 = parts[q].riv_recv_off[r], parts[q].riv_recv_off[r + 1]
            assert np.array_equal(p.riv_gid[p.riv_send_idx[s0:s1]],
                                  parts[q].riv_gid[parts[q].n_own_riv + d0:parts[q].n_own_riv + d1])
        p.close()


@SETTINGS
@given(n=st.integers(400, 3000), seed=st.integers(0, 10_000), nparts=st.integers(2, 5),
       mode=st.sampled_from([0, 1]))
def test_random_partition_simulation_bit_identical(n, seed, nparts, mode):
    """k ranks in one process (oracle RHS per local mesh, halo assembled from the peers' send buffers)."""
    import oracle
    from test_partition import _ghost_from_peers, _global_reach_order
    m, y = cases.variant(n, seed=seed)
    rng = np.random.default_rng(seed)
    ep = rng.integers(0, nparts, m.num_ele).astype(np.int32)
    ep[:nparts] = np.arange(nparts)
    locs = [partition.CppPlan(m, ep, nparts, r).local_model() for r in range(nparts)]
    parts = [p for _, p in locs]
    g = oracle.OracleRhs(m, mode)
    g.set_step_inputs()
    ors = []
    for lm, part in locs:
        lo, to_o, from_o = _global_reach_order(lm, part)
        o = oracle.OracleRhs(lo, mode)
        o.set_step_inputs()
        ors.append((o, to_o, from_o))
    for call in range(2):
        ref = g.eval(0.0, y)[0]
        owned = [partition.local_state(y, m, p) for p in parts]
        packs = [partition.pack_send(owned[r], parts[r]) for r in range(nparts)]
        for r, (lm, part) in enumerate(locs):
            gele, griv = _ghost_from_peers(parts, packs, r)
            o, to_o, from_o = ors[r]
            dy = from_o(o.eval(0.0, to_o(partition.extended_state(owned[r], gele, griv, part)))[0])
            assert np.array_equal(partition.owned_dy(dy, lm, part), partition.local_state(ref, m, part),
                                  equal_nan=True), (r, call)


@SETTINGS
@given(n=st.integers(500, 5000), seed=st.integers(0, 10_000), nparts=st.integers(2, 8))
def test_multilevel_partitioner_properties(n, seed, nparts):
    m, _ = cases.variant(n, seed=seed % 97)
    a, st_a = partition.cpp_partition(m, nparts, partition.PART_MULTILEVEL, seed=seed)
    b, _ = partition.cpp_partition(m, nparts, partition.PART_MULTILEVEL, seed=seed)
    assert np.array_equal(a, b)
    assert np.bincount(a, minlength=nparts).min() > 0
    w = 1.0 + np.bincount(m.seg_ele, minlength=m.num_ele)
    loads = np.bincount(a, weights=w, minlength=nparts)
    assert loads.max() / loads.mean() < 1.06          # 1.03 target + coarse-vertex granularity on small meshes
    assert (st_a["edge_cut"], st_a["segment_cut"]) == partition.edge_cut(m, a)
