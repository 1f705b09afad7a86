"""Seeded RHS workloads: states y and per-ET-step inputs (SURVEY §8c/§8d recipe).

States: y_sf = 0 w.p. 0.5 else U(0, 0.05); y_us = U(0, 0.5 Aq); y_gw = U(0, Aq); y_riv = U(0, 2).
Step inputs (units m, min as in SHUD): rates in the range an ET step of ccw produces (net precipitation
0-20 mm/day, PET 0-8 mm/day, LAI 0-4 with bare ground, interception evaporation below PET).
"""
import numpy as np


def random_state(model, seed=12345, n_own=None, n_own_riv=None):
    rng = np.random.default_rng(seed)
    NE = model.num_ele if n_own is None else n_own
    NR = model.num_riv if n_own_riv is None else n_own_riv
    aq = model.par["aquifer_depth"][:NE]
    sf = np.where(rng.random(NE) < 0.5, 0.0, rng.uniform(0.0, 0.05, NE))
    us = rng.uniform(0.0, 1.0, NE) * 0.5 * aq
    gw = rng.uniform(0.0, 1.0, NE) * aq
    rv = rng.uniform(0.0, 2.0, NR)
    lk = rng.uniform(0.0, 30.0, getattr(model, "num_lake", 0))     # lake stages (after the reaches)
    return np.concatenate([sf, us, gw, rv, lk])


def random_step_inputs(model, seed=777):
    rng = np.random.default_rng(seed)
    NE = model.num_ele
    day = 1.0 / 1440.0 / 1000.0          # mm/day -> m/min
    net_prep = np.where(rng.random(NE) < 0.4, 0.0, rng.uniform(0.0, 20.0, NE)) * day
    pot_evap = rng.uniform(0.0, 8.0, NE) * day
    pot_tran = rng.uniform(0.0, 6.0, NE) * day
    lai = np.where(rng.random(NE) < 0.2, 0.0, rng.uniform(0.0, 4.0, NE))
    e_ic = rng.uniform(0.0, 1.0, NE) * pot_tran * 1.2
    etp = pot_evap + pot_tran + rng.uniform(0.0, 1.0, NE) * day
    u_satn = rng.uniform(0.0, 1.0, NE)
    prcp = net_prep + rng.uniform(0.0, 5.0, NE) * day             # qElePrep (lake elements read it)
    return dict(net_prep=net_prep, pot_evap=pot_evap, pot_tran=pot_tran, etp=etp, lai=lai,
                fu_surf=np.ones(NE), fu_sub=np.ones(NE), e_ic=e_ic, u_satn=u_satn,
                ugw_stale=np.zeros(NE), prcp=prcp)
