"""GPU: partitioned handles (owned + ghost entities) on one MI355X, halo moved between the
handles' device buffers by the test (external transport: shud_rhs_eval_pack -> D2D copies ->
shud_rhs_eval_compute).  Owned DY must be bit-identical to the single-GPU handle's.  The RCCL transport
used by bench.py at N > 1 replaces only the D2D copies (grouped ncclSend/ncclRecv of the same ranges).

BASELINE configs[4] (syn-10M, 8-way partition, 8 GPUs) is exercised here as far as one GPU allows: the
8 partitioned handles of the bench's own C++ plan (include/shud_partition.h) live on one device and trade
their halos by D2D copies; every rank's owned DY equals the unpartitioned handle's bit for bit."""
import ctypes as C

import numpy as np
import pytest

import cases
from shud_rhs import abi, partition, workload

pytestmark = pytest.mark.gpu


def _run_ranks(m, y_list, locs, mode, ncalls=3, device_eval=False):
    """locs: [(local ShudModel, LocalPartition)] for every rank; compares owned DY with one unpartitioned
    handle over `ncalls` successive stateful calls per state."""
    from shud_rhs import runtime as rt
    nranks = len(locs)
    single = rt.RhsHandle(m, mode=mode)
    single.set_step_inputs()
    hs, bufs, halos = [], [], []
    try:
        for lm, part in locs:
            h = rt.RhsHandle(lm, mode=mode, partition=part)
            # a local mesh takes the same kernel layout as the whole mesh (ghosts' boundary-looking edges must
            # not push a rank onto the SoA kernel)
            assert h.layout()["packed"] == single.layout()["packed"], (h.layout(), single.layout())
            h.set_step_inputs()
            hs.append(h)
            ny = 3 * part.n_own_ele + part.n_own_riv + part.n_own_lake
            bufs.append((h.device_alloc(8 * ny), h.device_alloc(8 * ny), ny))
            halos.append(h.halo_buffers())
        # in-tile edge sharing (shud_rhs.cpp build_packed) covers a rank's interior prefix as well
        if single.layout().get("shared_edges"):
            assert sum(h.layout().get("shared_edges", 0) for h in hs) > 0, [h.layout() for h in hs]
        for yy in y_list:
            for call in range(ncalls):
                ref = single.eval(0.0, yy)
                for r, (lm, part) in enumerate(locs):
                    hs[r].h2d(bufs[r][0], partition.local_state(yy, m, part))
                    hs[r].eval_pack(bufs[r][0])
                    hs[r].synchronize()
                for r, (lm, part) in enumerate(locs):        # the all-to-all-v, as D2D copies
                    _, _, gele, griv = halos[r]
                    for p in range(nranks):
                        if p == r:
                            continue
                        esend, rsend, _, _ = halos[p]
                        pp = locs[p][1]
                        s0, s1 = int(pp.ele_send_off[r]), int(pp.ele_send_off[r + 1])
                        d0 = int(part.ele_recv_off[p])
                        assert s1 - s0 == int(part.ele_recv_off[p + 1]) - d0
                        if s1 > s0:
                            rt.lib().shud_rhs_memcpy(hs[r].h, C.c_void_p(gele + 24 * d0), C.c_void_p(esend + 24 * s0),
                                                     24 * (s1 - s0), 3)
                        s0, s1 = int(pp.riv_send_off[r]), int(pp.riv_send_off[r + 1])
                        d0 = int(part.riv_recv_off[p])
                        assert s1 - s0 == int(part.riv_recv_off[p + 1]) - d0
                        if s1 > s0:
                            rt.lib().shud_rhs_memcpy(hs[r].h, C.c_void_p(griv + 8 * d0), C.c_void_p(rsend + 8 * s0),
                                                     8 * (s1 - s0), 3)
                for r, (lm, part) in enumerate(locs):
                    if device_eval:     # the full device eval: pack + halo flag on the comm stream, folded launch
                        hs[r].eval_device(0.0, bufs[r][0], bufs[r][1])
                    else:
                        hs[r].eval_compute(0.0, bufs[r][0], bufs[r][1])
                    got = hs[r].d2h(np.zeros(bufs[r][2]), bufs[r][1])
                    if device_eval:
                        assert hs[r].get_error()["flags"] & 0x80 == 0, "SHUD_EF_HALO_WAIT"
                    want = partition.local_state(ref, m, part)
                    assert np.array_equal(got, want, equal_nan=True), f"rank {r} call {call}: {(got != want).sum()} differ"
    finally:
        for h, (a, b, _) in zip(hs, bufs):
            h.device_free(a)
            h.device_free(b)
            h.close()
        single.close()


@pytest.mark.parametrize("nranks", [2, 4, 8])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("packed", ["1", "0"])
def test_partitioned_handles_bit_identical(nranks, mode, packed, monkeypatch):
    """Python RCB plans (the restatement the C++ planner is checked against)."""
    monkeypatch.setenv("SHUD_RHS_PACKED", packed)
    m, y = cases.variant(20000, seed=17)
    _, _, plans = partition.build_plans(m, nranks)
    locs = [partition.local_model(m, plans[r], r, nranks) for r in range(nranks)]
    _run_ranks(m, [y, workload.random_state(m, seed=2)], locs, mode)


@pytest.mark.parametrize("fold", ["1", "0"])
@pytest.mark.parametrize("mode", [0, 1])
def test_device_eval_halo_flag(fold, mode, monkeypatch):
    """shud_rhs_eval on partitioned handles (external transport, halo placed by the test): the comm stream packs
    and publishes the halo epoch; with SHUD_RHS_FOLD=1 the boundary + ghost elements run in the interior launch and
    poll that flag, with 0 they are a second launch behind the comm event.  Both bit-identical to one GPU."""
    monkeypatch.setenv("SHUD_RHS_FOLD", fold)
    m, y = cases.variant(20000, seed=23)
    ep, _ = partition.cpp_partition(m, 4, partition.PART_AUTO)
    locs = [partition.CppPlan(m, ep, 4, r).local_model() for r in range(4)]
    _run_ranks(m, [y, workload.random_state(m, seed=8)], locs, mode, ncalls=2, device_eval=True)


@pytest.mark.parametrize("nranks", [2, 4, 8])
@pytest.mark.parametrize("method", [partition.PART_MULTILEVEL, partition.PART_AUTO])
def test_cpp_plans_bit_identical(nranks, method):
    """The C++ partitioner + planner + local-mesh gather (what bench.py N > 1 runs), serial and OMP."""
    m, y = cases.variant(20000, seed=17)
    ep, _ = partition.cpp_partition(m, nranks, method)
    locs = [partition.CppPlan(m, ep, nranks, r).local_model() for r in range(nranks)]
    for mode in (0, 1):
        _run_ranks(m, [y, workload.random_state(m, seed=5)], locs, mode, ncalls=2)


@pytest.mark.parametrize("device_eval", [False, True])
def test_hybrid_layout_partitions(device_eval):
    """Per-element-calibrated parameters (the hybrid layout: four class fields streamed per element) on 4 C++-planned
    ranks: every rank's local mesh chooses its own streamed fields and class table, and the owned DY stays
    bit-identical to the single GPU (a streamed value and a class-table value are the same bits; Sy's IEEE division
    equals the class reciprocal's cdiv)."""
    import test_gpu_parity as tp
    m, y = tp._hybrid_model(20000, seed=29)
    ep, _ = partition.cpp_partition(m, 4, partition.PART_AUTO)
    locs = [partition.CppPlan(m, ep, 4, r).local_model() for r in range(4)]
    for mode in (0, 1):
        _run_ranks(m, [y, workload.random_state(m, seed=6)], locs, mode, ncalls=2, device_eval=device_eval)


@pytest.mark.parametrize("nranks", [3, 5])
@pytest.mark.parametrize("seed", [2, 9])
def test_ragged_random_partitions(nranks, seed):
    """Random element-to-rank assignments (disconnected, ragged parts: every element can be a boundary element,
    every reach split) through the C++ planner: still bit-identical (NaNs of negative outlet stages included)."""
    m, y = cases.variant(6000, seed=seed)
    rng = np.random.default_rng(seed)
    ep = rng.integers(0, nranks, m.num_ele).astype(np.int32)
    ep[:nranks] = np.arange(nranks)
    locs = [partition.CppPlan(m, ep, nranks, r).local_model() for r in range(nranks)]
    for mode in (0, 1):
        _run_ranks(m, [y, workload.random_state(m, seed=seed + 1)], locs, mode, ncalls=2)


@pytest.mark.parametrize("case", ["qhh", "qhh_variant"])
@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_lake_partitions_bit_identical(case, nranks):
    """Lakes in partitioned handles: the C++ partitioner keeps each lake group (lake + bank
    elements) on one rank, which owns the lake stage and sums its terms in global order; reaches flowing into
    the lake (qhh_variant) are ghosts there when owned elsewhere.  Owned DY, lake stages included, must equal
    the single-GPU handle's bit for bit."""
    m, y = getattr(cases, case)()
    ep, _ = partition.cpp_partition(m, nranks, partition.PART_MULTILEVEL)
    locs = [partition.CppPlan(m, ep, nranks, r).local_model() for r in range(nranks)]
    assert sum(p.n_own_lake for _, p in locs) == m.num_lake
    _run_ranks(m, [y, workload.random_state(m, seed=3)], locs, 0, ncalls=2)


def test_lake_random_constrained_partition():
    """A ragged random partition of qhh_variant made lake-consistent by shud_partition_constrain."""
    m, y = cases.qhh_variant()
    rng = np.random.default_rng(11)
    ep = partition.cpp_constrain(m, rng.integers(0, 4, m.num_ele).astype(np.int32), 4)
    locs = [partition.CppPlan(m, ep, 4, r).local_model() for r in range(4)]
    _run_ranks(m, [y], locs, 0, ncalls=2)


@pytest.mark.parametrize("nranks,mode", [(2, 0), (8, 0), (4, 1)])
def test_syn_1m_cpp_plans(nranks, mode):
    """syn-1M (BASELINE configs[3] mesh) split by the bench's own C++ partition into 2, 4 and 8 ranks (serial
    semantics; OMP semantics at 4)."""
    from shud_rhs import synth
    m = synth.synth_model(1_000_000)
    m.step = workload.random_step_inputs(m)
    ep, _ = partition.cpp_partition(m, nranks, partition.PART_AUTO)
    locs = [partition.CppPlan(m, ep, nranks, r).local_model() for r in range(nranks)]
    _run_ranks(m, [workload.random_state(m)], locs, mode, ncalls=2)


def test_syn_10m_8way():
    """BASELINE configs[4]: syn-10M in the 8-way C++ partition the bench's N = 8 run uses, 8 partitioned
    handles on one GPU (D2D halo transport), 2 stateful calls: bit-identical to the single-GPU handle."""
    from shud_rhs import synth
    m = synth.synth_model(10_000_000)
    m.step = workload.random_step_inputs(m)
    ep, _ = partition.cpp_partition(m, 8, partition.PART_AUTO)
    locs = []
    for r in range(8):
        pl = partition.CppPlan(m, ep, 8, r)
        locs.append(pl.local_model())
        pl.close()
    _run_ranks(m, [workload.random_state(m)], locs, 0, ncalls=2)


@pytest.mark.parametrize("mode", [0, 1])
def test_rccl_comm_single_rank(mode):
    """The RCCL transport path (comm init from a unique id, comm stream + events, interior/boundary launch
    split) on a one-rank partition: must equal the unpartitioned handle bit for bit.  (N > 1 RCCL needs one
    GPU per rank; the multi-rank data movement itself is covered by the D2D-transport tests above.)"""
    from shud_rhs import runtime as rt
    m, y = cases.variant(20000, seed=17)
    single = rt.RhsHandle(m, mode=mode)
    single.set_step_inputs()
    _, _, plans = partition.build_plans(m, 1)
    lm, part = partition.local_model(m, plans[0], 0, 1)
    part.nccl_unique_id = rt.nccl_unique_id()
    h = rt.RhsHandle(lm, mode=mode, partition=part)
    h.set_step_inputs()
    ny = 3 * part.n_own_ele + part.n_own_riv
    dy_, ddy = h.device_alloc(8 * ny), h.device_alloc(8 * ny)
    try:
        for yy in [y, workload.random_state(m, seed=4)]:
            for call in range(3):
                ref = single.eval(0.0, yy)
                h.h2d(dy_, partition.local_state(yy, m, part))
                h.eval_device(0.0, dy_, ddy)
                got = h.d2h(np.zeros(ny), ddy)
                assert np.array_equal(got, partition.local_state(ref, m, part)), f"call {call}"
    finally:
        h.device_free(dy_)
        h.device_free(ddy)
        h.close()


def _late_halo_ranks(m, nranks):
    ep, _ = partition.cpp_partition(m, nranks, partition.PART_AUTO)
    return [partition.CppPlan(m, ep, nranks, r).local_model() for r in range(nranks)]


@pytest.mark.parametrize("mode", [0, 1])
def test_folded_halo_late(mode, monkeypatch):
    """The folded launch's halo hand-off with a genuinely LATE halo (VERDICT r03 item 2, MI355X guide: test every
    hand-off under uneven load, checking every word): each rank's comm stream spins ~200 us after its pack, then a
    kernel writes the ghost states (as RCCL's receive kernels would) and only then publishes the flag, so the boundary
    workgroups really poll while the interior workgroups run.  The ghost values change on every eval (a new state
    per call), so a stale line shows up; every owned DY word must equal the single handle's."""
    from shud_rhs import runtime as rt
    monkeypatch.setenv("SHUD_RHS_FOLD", "1")
    m, y = cases.variant(20000, seed=29)
    locs = _late_halo_ranks(m, 4)
    single = rt.RhsHandle(m, mode=mode)
    single.set_step_inputs()
    hs, bufs = [], []
    try:
        for lm, part in locs:
            h = rt.RhsHandle(lm, mode=mode, partition=part)
            h.set_step_inputs()
            ny = 3 * part.n_own_ele + part.n_own_riv
            ge, gr = partition.ghost_values(y, m, part)
            st_e, st_r = h.device_alloc(8 * max(1, ge.size)), h.device_alloc(8 * max(1, gr.size))
            bufs.append((h.device_alloc(8 * ny), h.device_alloc(8 * ny), ny, st_e, st_r))
            h.debug_halo(spin_us=200.0, d_ele_src=st_e, d_riv_src=st_r)
            hs.append(h)
        states = [workload.random_state(m, seed=100 + k) for k in range(6)]
        for call, yy in enumerate(states):            # a different state (and halo) on every stateful call
            ref = single.eval(0.0, yy)
            for r, (lm, part) in enumerate(locs):
                yb, dyb, ny, st_e, st_r = bufs[r]
                ge, gr = partition.ghost_values(yy, m, part)
                hs[r].h2d(yb, partition.local_state(yy, m, part))
                if ge.size:
                    hs[r].h2d(st_e, ge)
                if gr.size:
                    hs[r].h2d(st_r, gr)
                hs[r].eval_device(0.0, yb, dyb)
            for r, (lm, part) in enumerate(locs):
                yb, dyb, ny, _, _ = bufs[r]
                got = hs[r].d2h(np.zeros(ny), dyb)
                e = hs[r].get_error()
                assert e["flags"] & 0x80 == 0, f"rank {r} call {call}: SHUD_EF_HALO_WAIT"
                want = partition.local_state(ref, m, part)
                assert np.array_equal(got, want, equal_nan=True), \
                    f"rank {r} call {call}: {(~((got == want) | (np.isnan(got) & np.isnan(want)))).sum()} words differ"
    finally:
        for h, b in zip(hs, bufs):
            for p in (b[0], b[1], b[3], b[4]):
                h.device_free(p)
            h.close()
        single.close()


def test_folded_halo_never_arrives(monkeypatch):
    """The flag never comes: the boundary workgroups' bounded poll ends in the fatal SHUD_EF_HALO_WAIT and the eval
    returns an error (SHUD_ERR_PHYSICS); with the hook disarmed the next evals are bit-identical again."""
    from shud_rhs import runtime as rt
    monkeypatch.setenv("SHUD_RHS_FOLD", "1")
    m, y = cases.variant(20000, seed=31)
    lm, part = _late_halo_ranks(m, 2)[1]
    single = rt.RhsHandle(m)
    single.set_step_inputs()
    h = rt.RhsHandle(lm, partition=part)
    h.set_step_inputs()
    ge, gr = partition.ghost_values(y, m, part)
    st_e, st_r = h.device_alloc(8 * max(1, ge.size)), h.device_alloc(8 * max(1, gr.size))
    try:
        h.h2d(st_e, ge)
        h.h2d(st_r, gr)
        h.debug_halo(d_ele_src=st_e, d_riv_src=st_r, publish=False, timeout_ms=20.0)
        with pytest.raises(rt.ShudRhsError) as ei:
            h.eval(0.0, partition.local_state(y, m, part))
        assert ei.value.code == abi.SHUD_ERR_PHYSICS
        assert h.get_error()["flags"] & 0x80, "SHUD_EF_HALO_WAIT not raised"
        h.clear_error()
        # recovery: the flag is published again; both handles restart from the same step inputs / carried state
        h.debug_halo(d_ele_src=st_e, d_riv_src=st_r, publish=True)
        h.set_step_inputs()
        single.set_step_inputs()
        for call in range(2):
            ref = single.eval(0.0, y)
            got = h.eval(0.0, partition.local_state(y, m, part))
            assert np.array_equal(got, partition.local_state(ref, m, part), equal_nan=True), f"call {call}"
        assert h.get_error()["flags"] & 0x80 == 0
    finally:
        h.device_free(st_e)
        h.device_free(st_r)
        h.close()
        single.close()
