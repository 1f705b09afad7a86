"""Mesh partitioning and halo plans for one-process-per-GPU runs.

METIS is not available, so elements are split by weighted recursive coordinate bisection (RCB) of their
centroids (vertex weight 1 + number of river segments, as §8e asks of the dual-graph weight).  Ownership:
elements -> part; each reach -> the part owning most of its segments' elements (ties: lowest part; a reach
without segments follows its first element-owning neighbour reach, else part 0).

Local numbering of rank p:  elements [owned interior | owned boundary | ghosts grouped by source rank], each
group in global order (boundary = reads a ghost neighbour or a ghost reach; the interior runs during the halo exchange),
reaches [owned | ghosts grouped by source rank], segments = every segment whose element or reach is owned,
in global segment order.  Ghost elements = lateral neighbours of owned elements + elements of segments of
owned reaches; they carry replicated static data, step inputs and carried state, and the element kernel
recomputes their vertical/segment fluxes (never their DY).  Ghost reaches = reaches of owned elements'
segments + downstream and upstream reaches of owned reaches.  One exchange per RHS ships the ghost states.
Because every owned value is computed exactly as on one GPU, with reductions in global order, partitioned
results are bit-identical to the single-GPU result.
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List

import numpy as np

from . import abi
from .model import ELE1, ELE3, RIV_D, ShudModel


def rcb(x, y, w, nparts):
    """Weighted recursive coordinate bisection -> part id per point (0..nparts-1)."""
    part = np.zeros(x.size, dtype=np.int32)

    def rec(idx, p0, np_):
        if np_ == 1 or idx.size == 0:
            part[idx] = p0
            return
        nl = np_ // 2
        xs, ys = x[idx], y[idx]
        key = xs if (xs.max() - xs.min()) >= (ys.max() - ys.min()) else ys
        order = np.argsort(key, kind="stable")
        cw = np.cumsum(w[idx][order])
        cut = np.searchsorted(cw, cw[-1] * nl / np_)
        cut = min(max(cut, 1), idx.size - 1) if idx.size > 1 else 0
        rec(np.sort(idx[order[:cut]]), p0, nl)
        rec(np.sort(idx[order[cut:]]), p0 + nl, np_ - nl)

    rec(np.arange(x.size), 0, nparts)
    return part


def element_centroids(m):
    if "x" in m.meta and "y" in m.meta:
        return np.asarray(m.meta["x"]), np.asarray(m.meta["y"])
    raise ValueError("model has no element centroids (meta x/y)")


def assign_owners(m, nparts, ele_part=None):
    if ele_part is None:
        x, y = element_centroids(m)
        w = 1.0 + np.bincount(m.seg_ele, minlength=m.num_ele)
        ele_part = rcb(x, y, w, nparts)
    NR = m.num_riv
    cnt = np.zeros((NR, nparts), dtype=np.int64)
    np.add.at(cnt, (m.seg_riv, ele_part[m.seg_ele]), 1)
    riv_part = np.argmax(cnt, axis=1).astype(np.int32)      # argmax: lowest part on ties
    noseg = cnt.sum(1) == 0
    riv_part[noseg] = 0
    return ele_part.astype(np.int32), riv_part


@dataclass
class LocalPartition:
    rank: int
    nranks: int
    n_own_ele: int
    n_own_riv: int
    ele_gid: np.ndarray
    riv_gid: np.ndarray
    ele_send_off: np.ndarray
    ele_send_idx: np.ndarray
    ele_recv_off: np.ndarray
    riv_send_off: np.ndarray
    riv_send_idx: np.ndarray
    riv_recv_off: np.ndarray
    seg_gid: np.ndarray
    nccl_unique_id: bytes = None
    lake_gid: np.ndarray = None            # owned lakes (0-based global ids), C++ plans only
    _keep: List = field(default_factory=list)

    @property
    def n_segghost_ele(self):
        return self.ele_gid.size - self.n_own_ele

    @property
    def n_own_lake(self):
        return 0 if self.lake_gid is None else int(self.lake_gid.size)

    def struct(self):
        p = abi.ShudPartition()
        p.rank, p.nranks = self.rank, self.nranks
        p.n_own_ele, p.n_segghost_ele, p.n_own_riv = self.n_own_ele, self.n_segghost_ele, self.n_own_riv
        arrs = {}
        for k in ["ele_send_off", "ele_send_idx", "ele_recv_off", "riv_send_off", "riv_send_idx", "riv_recv_off",
                  "ele_gid", "riv_gid"]:
            a = np.ascontiguousarray(getattr(self, k), dtype=np.int32)
            arrs[k] = a
            setattr(p, k, a.ctypes.data_as(abi.c_int32_p))
        p.nccl_unique_id = self.nccl_unique_id
        self._keep = [arrs, p]
        return p


def _ghost_sets(m, ele_part, riv_part, r):
    own_e = np.nonzero(ele_part == r)[0]
    own_r = np.nonzero(riv_part == r)[0]
    own_e_mask = ele_part == r
    own_r_mask = riv_part == r
    seg_mask = own_e_mask[m.seg_ele] | own_r_mask[m.seg_riv]
    segs = np.nonzero(seg_mask)[0]
    nab = m.nabr.reshape(3, -1)[:, own_e].reshape(-1)
    nab = nab[nab >= 0]
    ghost_e = np.union1d(nab, m.seg_ele[segs])
    ghost_e = ghost_e[~own_e_mask[ghost_e]]
    rd = m.riv_down[own_r]
    up = np.nonzero((m.riv_down >= 0) & own_r_mask[np.where(m.riv_down >= 0, m.riv_down, 0)])[0]
    ghost_r = np.union1d(np.union1d(m.seg_riv[segs], rd[rd >= 0]), up)
    ghost_r = ghost_r[~own_r_mask[ghost_r]]
    # owned elements: [interior | boundary] (stable).  Boundary = reads ghost data: a lateral neighbour or a
    # segment reach owned elsewhere.  The interior prefix runs while the halo exchange is in flight.
    nb = m.nabr.reshape(3, -1)[:, own_e]
    dep = ((nb >= 0) & ~own_e_mask[np.where(nb >= 0, nb, 0)]).any(axis=0)
    own_seg = own_e_mask[m.seg_ele]
    bad_seg_ele = m.seg_ele[own_seg & ~own_r_mask[m.seg_riv]]
    dep |= np.isin(own_e, bad_seg_ele)
    own_e = np.concatenate([own_e[~dep], own_e[dep]])
    return own_e, own_r, segs, ghost_e, ghost_r


def edge_cut(m, ele_part):
    """Partition quality: #mesh edges whose two elements are on different parts, and #river
    segments whose element and reach are owned by different parts."""
    nab = m.nabr.reshape(3, -1)
    i = np.broadcast_to(np.arange(m.num_ele), nab.shape)
    ok = nab > i                          # each interior edge once
    cut_e = int((ele_part[i[ok]] != ele_part[nab[ok]]).sum())
    _, riv_part = assign_owners(m, int(ele_part.max()) + 1, ele_part)
    cut_s = int((ele_part[m.seg_ele] != riv_part[m.seg_riv]).sum())
    return cut_e, cut_s


def build_plans(m, nparts, ele_part=None):
    """Global partition -> per-rank (local element order, local reach order, segment set, plan)."""
    ele_part, riv_part = assign_owners(m, nparts, ele_part)
    sets = [_ghost_sets(m, ele_part, riv_part, r) for r in range(nparts)]
    orders = []
    for r in range(nparts):
        own_e, own_r, segs, ge, gr = sets[r]
        # ghosts grouped by source rank, global order inside a group (stable sort)
        ge = ge[np.argsort(ele_part[ge], kind="stable")]
        gr = gr[np.argsort(riv_part[gr], kind="stable")]
        orders.append((own_e, own_r, segs, ge, gr))
    plans = []
    for r in range(nparts):
        own_e, own_r, segs, ge, gr = orders[r]
        erecv = np.zeros(nparts + 1, dtype=np.int64)
        rrecv = np.zeros(nparts + 1, dtype=np.int64)
        erecv[1:] = np.cumsum(np.bincount(ele_part[ge], minlength=nparts))
        rrecv[1:] = np.cumsum(np.bincount(riv_part[gr], minlength=nparts))
        # what r sends to q = the ghosts q receives from r, in q's order
        esend_idx, rsend_idx = [], []
        esend = np.zeros(nparts + 1, dtype=np.int64)
        rsend = np.zeros(nparts + 1, dtype=np.int64)
        g2l_e = np.full(m.num_ele, -1, dtype=np.int64)
        g2l_e[own_e] = np.arange(own_e.size)
        g2l_r = np.full(m.num_riv, -1, dtype=np.int64)
        g2l_r[own_r] = np.arange(own_r.size)
        for q in range(nparts):
            if q == r:
                esend[q + 1] = esend[q]
                rsend[q + 1] = rsend[q]
                continue
            _, _, _, geq, grq = orders[q]
            ee = geq[ele_part[geq] == r]
            rr = grq[riv_part[grq] == r]
            esend_idx.append(g2l_e[ee])
            rsend_idx.append(g2l_r[rr])
            esend[q + 1] = esend[q] + ee.size
            rsend[q + 1] = rsend[q] + rr.size
        plans.append(dict(own_e=own_e, own_r=own_r, segs=segs, ghost_e=ge, ghost_r=gr, erecv=erecv, rrecv=rrecv,
                          esend=esend, rsend=rsend,
                          esend_idx=np.concatenate(esend_idx) if esend_idx else np.zeros(0, dtype=np.int64),
                          rsend_idx=np.concatenate(rsend_idx) if rsend_idx else np.zeros(0, dtype=np.int64)))
    return ele_part, riv_part, plans


def local_model(m, plan, rank, nranks):
    """Extract rank's local ShudModel (owned + ghosts) and its LocalPartition."""
    own_e, own_r, segs, ge, gr = plan["own_e"], plan["own_r"], plan["segs"], plan["ghost_e"], plan["ghost_r"]
    le = np.concatenate([own_e, ge])
    lr = np.concatenate([own_r, gr])
    NE, NR = le.size, lr.size
    g2l_e = np.full(m.num_ele, -1, dtype=np.int64)
    g2l_e[le] = np.arange(NE)
    g2l_r = np.full(m.num_riv, -1, dtype=np.int64)
    g2l_r[lr] = np.arange(NR)
    lm = ShudModel(NE, NR, segs.size, m.close_boundary)
    for k in ELE1:
        if k in m.ele:
            lm.ele[k] = m.ele[k][le]
    for k in ELE3:
        if k in m.ele:
            lm.ele[k] = m.ele[k].reshape(3, -1)[:, le].reshape(-1)
    nab = m.nabr.reshape(3, -1)[:, le]
    lm.nabr = np.where(nab >= 0, g2l_e[np.where(nab >= 0, nab, 0)], -1).reshape(-1)
    lm.ibc = m.ibc[le]
    lm.iss = m.iss[le]
    if m.ilake is not None:
        lm.ilake = m.ilake[le]
    for k in RIV_D:
        lm.riv[k] = m.riv[k][lr]
    d = m.riv_down[lr]
    dl = np.where(d >= 0, g2l_r[np.where(d >= 0, d, 0)], d)
    lm.riv_down = np.where((d >= 0) & (dl < 0), -3, dl)      # downstream outside this rank: never used
    lm.riv_bc = m.riv_bc[lr]
    lm.seg_ele = g2l_e[m.seg_ele[segs]]
    lm.seg_riv = g2l_r[m.seg_riv[segs]]
    lm.seg_length = m.seg_length[segs]
    lm.seg_cwr = m.seg_cwr[segs]
    for k in abi.PARAM_NAMES:
        lm.par[k] = m.par[k][le]
    for k, v in m.step.items():
        lm.step[k] = v[le]
    lm.bc_tables = dict(m.bc_tables)
    lm.meta["ele_gid"] = le
    lm.meta["riv_gid"] = lr
    lm.finalize()
    part = LocalPartition(rank=rank, nranks=nranks, n_own_ele=own_e.size, n_own_riv=own_r.size,
                          ele_gid=le, riv_gid=lr, ele_send_off=plan["esend"], ele_send_idx=plan["esend_idx"],
                          ele_recv_off=plan["erecv"], riv_send_off=plan["rsend"], riv_send_idx=plan["rsend_idx"],
                          riv_recv_off=plan["rrecv"], seg_gid=segs)
    return lm, part


def local_state(y_global, m_global, part):
    """Owned part of a global state vector in the rank's reference block layout [sf|us|gw|riv|lake]."""
    NE, NR = m_global.num_ele, m_global.num_riv
    oe = part.ele_gid[:part.n_own_ele]
    orr = part.riv_gid[:part.n_own_riv]
    ol = part.lake_gid if part.lake_gid is not None else np.zeros(0, np.int64)
    return np.concatenate([y_global[oe], y_global[NE + oe], y_global[2 * NE + oe], y_global[3 * NE + orr],
                           y_global[3 * NE + NR + ol]])


def ghost_values(y_global, m_global, part):
    """Ghost buffers as the exchange delivers them (ele AoS [sf,us,gw], reaches) — for tests."""
    NE = m_global.num_ele
    ge = part.ele_gid[part.n_own_ele:]
    gr = part.riv_gid[part.n_own_riv:]
    ele = np.stack([y_global[ge], y_global[NE + ge], y_global[2 * NE + ge]], 1).reshape(-1)
    return ele, y_global[3 * NE + gr]


def extended_state(y_owned, gele, griv, part):
    """[sf|us|gw|riv|lake] over ALL local entities (owned + ghost; lakes are always owned): the CPU oracle's
    input for a rank."""
    no, nro, nl = part.n_own_ele, part.n_own_riv, part.n_own_lake
    g = gele.reshape(-1, 3)
    sf = np.concatenate([y_owned[:no], g[:, 0]])
    us = np.concatenate([y_owned[no:2 * no], g[:, 1]])
    gw = np.concatenate([y_owned[2 * no:3 * no], g[:, 2]])
    rv = np.concatenate([y_owned[3 * no:3 * no + nro], griv])
    return np.concatenate([sf, us, gw, rv, y_owned[3 * no + nro:3 * no + nro + nl]])


def owned_dy(dy_ext, lm, part):
    """Owned entries of an extended-layout ydot, in the owned block layout."""
    NEl, NRl, no, nro, nl = lm.num_ele, lm.num_riv, part.n_own_ele, part.n_own_riv, part.n_own_lake
    return np.concatenate([dy_ext[:no], dy_ext[NEl:NEl + no], dy_ext[2 * NEl:2 * NEl + no],
                           dy_ext[3 * NEl:3 * NEl + nro], dy_ext[3 * NEl + NRl:3 * NEl + NRl + nl]])


def pack_send(y_owned, part):
    """CPU equivalent of shud_pack_kernel: ele AoS records and reach values for all peers."""
    no = part.n_own_ele
    i = np.asarray(part.ele_send_idx, dtype=np.int64)
    ebuf = np.stack([y_owned[i], y_owned[no + i], y_owned[2 * no + i]], 1).reshape(-1)
    rbuf = y_owned[3 * no + np.asarray(part.riv_send_idx, dtype=np.int64)]
    return ebuf, rbuf


# ---------------------------------------------------------------------------------------------------------
# The C++ partitioner and planner (include/shud_partition.h, libshud_host.so).  The functions above are the
# Python restatement the tests cross-check it against; bench.py's N > 1 path uses the C++ ones.
# ---------------------------------------------------------------------------------------------------------
PART_MULTILEVEL, PART_RCB, PART_AUTO = 0, 1, 2


class ShudPartStats(C.Structure):
    _fields_ = [("edge_cut", C.c_int64), ("segment_cut", C.c_int64), ("graph_cut", C.c_int64),
                ("imbalance", C.c_double), ("levels", C.c_int32), ("coarse_vertices", C.c_int32),
                ("seconds", C.c_double), ("max_halo", C.c_int64), ("method_used", C.c_int32)]


class ShudPlanInfo(C.Structure):
    _fields_ = [("n_own_ele", C.c_int32), ("n_int_ele", C.c_int32), ("n_ghost_ele", C.c_int32),
                ("n_own_riv", C.c_int32), ("n_ghost_riv", C.c_int32), ("n_seg", C.c_int32),
                ("ele_gid", C.POINTER(C.c_int32)), ("riv_gid", C.POINTER(C.c_int32)),
                ("seg_gid", C.POINTER(C.c_int32)), ("riv_part", C.POINTER(C.c_int32)),
                ("n_own_lake", C.c_int32), ("lake_gid", C.POINTER(C.c_int32))]


_HL = None


def _host():
    global _HL
    if _HL is None:
        from . import host
        L = host.lib()
        H = C.c_void_p
        sig = {
            "shud_partition_mesh": (C.c_int, [C.POINTER(abi.ShudMeshSoA), C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                              C.c_uint64, C.c_void_p, C.POINTER(ShudPartStats)]),
            "shud_partition_constrain": (C.c_int, [C.POINTER(abi.ShudMeshSoA), C.c_int32, C.c_void_p]),
            "shud_partition_cut": (C.c_int, [C.POINTER(abi.ShudMeshSoA), C.c_void_p, C.c_int32,
                                             C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
            "shud_partition_halo": (C.c_int, [C.POINTER(abi.ShudMeshSoA), C.c_void_p, C.c_int32, C.c_void_p,
                                              C.c_void_p]),
            "shud_plan_build": (C.c_int, [C.POINTER(abi.ShudMeshSoA), C.c_void_p, C.c_int32, C.c_int32,
                                          C.POINTER(H)]),
            "shud_plan_free": (None, [H]),
            "shud_plan_info": (C.c_int, [H, C.POINTER(ShudPlanInfo)]),
            "shud_plan_partition": (C.c_int, [H, C.POINTER(abi.ShudPartition)]),
            "shud_plan_local_mesh": (C.c_int, [H, C.POINTER(abi.ShudMeshSoA), C.POINTER(abi.ShudParamsSoA),
                                               C.POINTER(abi.ShudMeshSoA), C.POINTER(abi.ShudParamsSoA)]),
            "shud_plan_gather_ele": (C.c_int, [H, C.c_void_p, C.c_void_p]),
            "shud_plan_owned_state": (C.c_int, [H, C.c_void_p, C.c_int32, C.c_void_p]),
            "shud_plan_scatter_owned": (C.c_int, [H, C.c_void_p, C.c_int32, C.c_void_p]),
            "shud_partition_error": (C.c_char_p, []),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _HL = L
    return _HL


def _hcheck(rc, what):
    if rc:
        raise RuntimeError(f"{what} failed ({rc}): {_host().shud_partition_error().decode()}")


def cpp_partition(m, nparts, method=PART_MULTILEVEL, seed=12345):
    """C++ element partition (multilevel HEM + FM/greedy refinement, or RCB) -> (ele_part, stats dict)."""
    ms = m.mesh_struct()
    part = np.zeros(m.num_ele, dtype=np.int32)
    cx = cy = None
    if method in (PART_RCB, PART_AUTO) and "x" in m.meta:
        x, y = element_centroids(m)
        cx, cy = np.ascontiguousarray(x, dtype=np.float64), np.ascontiguousarray(y, dtype=np.float64)
    st = ShudPartStats()
    _hcheck(_host().shud_partition_mesh(C.byref(ms), None if cx is None else cx.ctypes.data,
                                        None if cy is None else cy.ctypes.data, int(nparts), int(method),
                                        int(seed), part.ctypes.data, C.byref(st)), "shud_partition_mesh")
    stats = {k: getattr(st, k) for k, _ in ShudPartStats._fields_}
    return part, stats


def cpp_constrain(m, ele_part, nparts):
    """A caller's partition with every lake group moved onto one part (shud_partition_constrain)."""
    ms = m.mesh_struct()
    ep = np.array(ele_part, dtype=np.int32)
    _hcheck(_host().shud_partition_constrain(C.byref(ms), int(nparts), ep.ctypes.data), "shud_partition_constrain")
    return ep


def cpp_edge_cut(m, ele_part):
    ms = m.mesh_struct()
    ep = np.ascontiguousarray(ele_part, dtype=np.int32)
    ec, sc = C.c_int64(), C.c_int64()
    _hcheck(_host().shud_partition_cut(C.byref(ms), ep.ctypes.data, int(ep.max()) + 1, C.byref(ec), C.byref(sc)),
            "shud_partition_cut")
    return ec.value, sc.value


def cpp_halo(m, ele_part):
    """(ghost elements, ghost reaches) per part, from the C++ planner's ownership rules"""
    ms = m.mesh_struct()
    ep = np.ascontiguousarray(ele_part, dtype=np.int32)
    k = int(ep.max()) + 1
    ge, gr = np.zeros(k, np.int64), np.zeros(k, np.int64)
    _hcheck(_host().shud_partition_halo(C.byref(ms), ep.ctypes.data, k, ge.ctypes.data, gr.ctypes.data),
            "shud_partition_halo")
    return ge, gr


class CppPlan:
    """One rank's plan built by the C++ planner (shud_plan_build); .local_model() = the rank's ShudModel and
    LocalPartition gathered by C++ (shud_plan_local_mesh / shud_plan_gather_ele)."""

    def __init__(self, m, ele_part, nparts, rank):
        self.m = m
        self.nparts, self.rank = nparts, rank
        self._ms = m.mesh_struct()
        self._ep = np.ascontiguousarray(ele_part, dtype=np.int32)
        h = C.c_void_p()
        _hcheck(_host().shud_plan_build(C.byref(self._ms), self._ep.ctypes.data, int(nparts), int(rank),
                                        C.byref(h)), "shud_plan_build")
        self.h = h
        info = ShudPlanInfo()
        _hcheck(_host().shud_plan_info(h, C.byref(info)), "shud_plan_info")
        ne, nr = info.n_own_ele + info.n_ghost_ele, info.n_own_riv + info.n_ghost_riv
        self.n_own_ele, self.n_int_ele, self.n_own_riv = info.n_own_ele, info.n_int_ele, info.n_own_riv
        self.ele_gid = np.ctypeslib.as_array(info.ele_gid, shape=(ne,)).copy()
        self.riv_gid = np.ctypeslib.as_array(info.riv_gid, shape=(nr,)).copy()
        self.seg_gid = (np.ctypeslib.as_array(info.seg_gid, shape=(info.n_seg,)).copy() if info.n_seg
                        else np.zeros(0, np.int32))
        self.riv_part = (np.ctypeslib.as_array(info.riv_part, shape=(m.num_riv,)).copy() if m.num_riv
                         else np.zeros(0, np.int32))
        self.lake_gid = (np.ctypeslib.as_array(info.lake_gid, shape=(info.n_own_lake,)).copy() if info.n_own_lake
                         else np.zeros(0, np.int32))
        sp = abi.ShudPartition()
        _hcheck(_host().shud_plan_partition(h, C.byref(sp)), "shud_plan_partition")
        P = nparts + 1

        def arr(ptr, n):
            return np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n else np.zeros(0, np.int32)
        self.ele_send_off = arr(sp.ele_send_off, P)
        self.ele_recv_off = arr(sp.ele_recv_off, P)
        self.riv_send_off = arr(sp.riv_send_off, P)
        self.riv_recv_off = arr(sp.riv_recv_off, P)
        self.ele_send_idx = arr(sp.ele_send_idx, int(self.ele_send_off[-1]))
        self.riv_send_idx = arr(sp.riv_send_idx, int(self.riv_send_off[-1]))

    def close(self):
        if self.h:
            _host().shud_plan_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def partition(self):
        return LocalPartition(rank=self.rank, nranks=self.nparts, n_own_ele=self.n_own_ele, n_own_riv=self.n_own_riv,
                              ele_gid=self.ele_gid, riv_gid=self.riv_gid, ele_send_off=self.ele_send_off,
                              ele_send_idx=self.ele_send_idx, ele_recv_off=self.ele_recv_off,
                              riv_send_off=self.riv_send_off, riv_send_idx=self.riv_send_idx,
                              riv_recv_off=self.riv_recv_off, seg_gid=self.seg_gid, lake_gid=self.lake_gid)

    def gather_ele(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        out = np.empty(self.ele_gid.size)
        _hcheck(_host().shud_plan_gather_ele(self.h, a.ctypes.data, out.ctypes.data), "shud_plan_gather_ele")
        return out

    def owned_state(self, y):
        y = np.ascontiguousarray(y, dtype=np.float64)
        out = np.empty(3 * self.n_own_ele + self.n_own_riv + self.lake_gid.size)
        _hcheck(_host().shud_plan_owned_state(self.h, y.ctypes.data, self.m.num_ele, out.ctypes.data),
                "shud_plan_owned_state")
        return out

    def local_model(self):
        """(ShudModel, LocalPartition) of this rank, every array gathered by the C++ planner."""
        m = self.m
        lms, lps = abi.ShudMeshSoA(), abi.ShudParamsSoA()
        gps = m.params_struct()
        _hcheck(_host().shud_plan_local_mesh(self.h, C.byref(self._ms), C.byref(gps), C.byref(lms), C.byref(lps)),
                "shud_plan_local_mesh")
        NE, NR, NS = lms.num_ele, lms.num_riv, lms.num_seg

        def d(ptr, n):
            return np.ctypeslib.as_array(ptr, shape=(n,)).copy() if (ptr and n) else None
        lm = ShudModel(NE, NR, NS, lms.close_boundary)
        for k in ELE1:
            v = d(getattr(lms, k), NE)
            if v is not None:
                lm.ele[k] = v
        for k in ELE3:
            v = d(getattr(lms, k), 3 * NE)
            if v is not None:
                lm.ele[k] = v
        lm.nabr = d(lms.nabr, 3 * NE)
        lm.ibc, lm.iss = d(lms.ibc, NE), d(lms.iss, NE)
        lm.ilake = d(lms.ilake, NE)
        if lms.num_lake > 0:
            nl = lms.num_lake
            lm.num_lake = nl
            lm.lake_bathy_off = d(lms.lake_bathy_off, nl + 1)
            nb = int(lm.lake_bathy_off[-1])
            lm.lake_bathy_y, lm.lake_bathy_a = d(lms.lake_bathy_y, nb), d(lms.lake_bathy_a, nb)
        for k in RIV_D:
            v = d(getattr(lms, k), NR)
            lm.riv[k] = v if v is not None else np.zeros(NR)
        lm.riv_down = d(lms.riv_down, NR) if NR else np.zeros(0, np.int32)
        lm.riv_bc = d(lms.riv_bc, NR) if NR else np.zeros(0, np.int32)
        lm.seg_ele = d(lms.seg_ele, NS) if NS else np.zeros(0, np.int32)
        lm.seg_riv = d(lms.seg_riv, NS) if NS else np.zeros(0, np.int32)
        lm.seg_length = d(lms.seg_length, NS) if NS else np.zeros(0)
        lm.seg_cwr = d(lms.seg_cwr, NS) if NS else np.zeros(0)
        for k in abi.PARAM_NAMES:
            lm.par[k] = d(getattr(lps, k), NE)
        for k, v in m.step.items():
            lm.step[k] = self.gather_ele(v)
        lm.bc_tables = dict(m.bc_tables)
        lm.meta["ele_gid"] = self.ele_gid
        lm.meta["riv_gid"] = self.riv_gid
        lm.finalize()
        return lm, self.partition()
