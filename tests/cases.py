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
