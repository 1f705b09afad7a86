"""Shared parity cases: reference inputs (ccw, heihe) and a synthetic variant that exercises the branches
no shipped input touches (open boundary, bank slope > 0, element/river BCs, source/sink flags, every
outlet code) — SURVEY §8c "F3 synthetic"."""
import numpy as np

from conftest import load_fixture
from shud_rhs import synth, workload


def ccw():
    m, y0 = load_fixture("ccw")
    m.step = workload.random_step_inputs(m, seed=11)
    return m, y0


def heihe():
    m, y0 = load_fixture("heihe")
    m.step = workload.random_step_inputs(m, seed=12)
    return m, y0


def qhh():
    """qhh: 4773 elements, 688 of them in one lake (.lake.bathy), bank edges around it."""
    m, y0 = load_fixture("qhh")
    m.step = workload.random_step_inputs(m, seed=13)
    return m, y0


def qhh_variant(seed=7):
    """qhh with a few outlet reaches redirected into the lake (down = -4: toLake 0, MD_Lake.cpp:46-50),
    fu != 1 and a low lake stage (exercises the 0.02 m dry guards and the qLakeEvap clamp)."""
    m, y0 = load_fixture("qhh")
    rng = np.random.default_rng(seed)
    outs = np.nonzero(m.riv_down < 0)[0]
    m.riv_down[outs[::3]] = -4
    m.step = workload.random_step_inputs(m, seed=seed)
    m.step["fu_surf"] = rng.uniform(0.5, 1.0, m.num_ele)
    m.step["fu_sub"] = rng.uniform(0.5, 1.0, m.num_ele)
    m.finalize()
    y = workload.random_state(m, seed=seed + 1)
    y[-1] = 0.01
    return m, y


def variant(n=2000, seed=5):
    """Synthetic mesh with CLOSEBOUNDARY 0, bank slopes, +-BC elements/reaches, SS flags, outlets."""
    m = synth.synth_model(n, seed=seed)
    rng = np.random.default_rng(seed)
    NE, NR = m.num_ele, m.num_riv
    m.close_boundary = 0
    m.riv["riv_bankslope"] = np.where(rng.random(NR) < 0.6, rng.uniform(0.1, 2.0, NR), 0.0)
    ibc = np.zeros(NE, dtype=np.int32)
    k = rng.choice(NE, 40, replace=False)
    ibc[k[:20]] = rng.integers(1, 3, 20)            # fixed head, columns 1..2
    ibc[k[20:]] = -rng.integers(1, 4, 20)           # fixed flux, columns 1..3
    m.ibc = ibc
    iss = np.zeros(NE, dtype=np.int32)
    iss[rng.choice(NE, 30, replace=False)] = rng.choice([-1, 1], 30)
    m.iss = iss
    rbc = np.zeros(NR, dtype=np.int32)
    kr = rng.choice(NR, 12, replace=False)
    rbc[kr[:6]] = 1
    rbc[kr[6:]] = -rng.integers(1, 3, 6)
    m.riv_bc = rbc
    outs = np.nonzero(m.riv_down < 0)[0]
    codes = np.array([-1, -2, -3, -4])
    m.riv_down[outs] = codes[np.arange(outs.size) % 4]
    m.step = workload.random_step_inputs(m, seed=seed + 1)
    m.step["ugw_stale"] = rng.uniform(0.0, 20.0, NE)
    m.step["fu_surf"] = rng.uniform(0.5, 1.0, NE)
    m.step["fu_sub"] = rng.uniform(0.5, 1.0, NE)
    m.bc_tables = dict(ele_ybc=np.array([0.0, 12.5, 25.0]), ele_qbc=np.array([0.0, -3.0, 5.0, 0.25]),
                       riv_ybc=np.array([0.0, 0.8]), riv_qbc=np.array([0.0, 2.0, -1.5]))
    m.finalize()
    y = workload.random_state(m, seed=seed + 2)
    # a few negative states (serial mode passes them unclamped, OMP clamps)
    neg = rng.choice(m.num_y, 30, replace=False)
    y[neg] = -np.abs(y[neg]) * 0.01
    return m, y


def states(m, y0=None, n_random=4, seed=100):
    out = [] if y0 is None else [y0]
    for k in range(n_random):
        out.append(workload.random_state(m, seed=seed + k))
    return out


def _subset(m, keep, close_boundary=None):
    """elements `keep` of m (neighbours outside become boundary edges), no rivers"""
    from shud_rhs import ShudModel
    keep = np.asarray(keep)
    NE = m.num_ele
    g2l = np.full(NE, -1, dtype=np.int64)
    g2l[keep] = np.arange(keep.size)
    r = ShudModel(keep.size, 0, 0, m.close_boundary if close_boundary is None else close_boundary)
    for k, v in m.ele.items():
        r.ele[k] = v.reshape(3, -1)[:, keep].reshape(-1) if v.size == 3 * NE else v[keep]
    nab = m.nabr.reshape(3, -1)[:, keep]
    r.nabr = np.where(nab >= 0, g2l[np.where(nab >= 0, nab, 0)], -1).reshape(-1).astype(np.int32)
    # an edge whose neighbour was dropped is a boundary edge: avgRough = the element's own Rough there
    # (Element.cpp:249-265)
    cut = (r.nabr.reshape(3, -1) < 0) & (nab >= 0)
    ar = r.ele["avg_rough"].reshape(3, -1).copy()
    ar[cut] = np.broadcast_to(r.ele["rough"], ar.shape)[cut]
    r.ele["avg_rough"] = ar.reshape(-1)
    r.ibc, r.iss = m.ibc[keep], m.iss[keep]
    r.par = {k: v[keep] for k, v in m.par.items()}
    r.step = {k: v[keep] for k, v in m.step.items()}
    r.riv = {}
    r.riv_down = np.zeros(0, np.int32)
    r.riv_bc = np.zeros(0, np.int32)
    r.seg_ele = np.zeros(0, np.int32)
    r.seg_riv = np.zeros(0, np.int32)
    r.seg_length = np.zeros(0)
    r.seg_cwr = np.zeros(0)
    return r.finalize()


def riverless():
    """ccw without its river network (NR = NS = 0): element fluxes only."""
    m, y0 = ccw()
    return _subset(m, np.arange(m.num_ele)), y0[:3 * m.num_ele].copy()


def single_element(close_boundary=0):
    """one triangle, every edge a domain boundary (the open-boundary outflow of MD_ElementFlux.cpp:81-93,
    139-152 on all three edges when close_boundary = 0)."""
    m, y0 = ccw()
    r = _subset(m, np.array([5]), close_boundary)
    y = np.array([0.03, 0.4 * r.par["aquifer_depth"][0], 0.6 * r.par["aquifer_depth"][0]])
    return r, y
