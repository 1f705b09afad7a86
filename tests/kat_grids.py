"""Edge-case input grids for the leaf-equation known-answer tests.

Each grid crosses every branch boundary of its reference function (values at, just below and just above
each threshold: ZERO = 1e-10, EPSILON = 0.005, EPS_SLOPE = 5e-8, 0.99, field capacity) plus a seeded random
cloud.  Ids and argument order follow oracle_kat() (oracle/shud_oracle.c) and shud_kat.hip."""
import itertools

import numpy as np

KAT = dict(MANNING=0, EFFKH=1, WEIR=2, R2E=3, SATK=4, SMS=5, DADY=6, AREA=7, PEREM=8, TOPW=9, TOPAREA=10)
NIN = [4, 6, 8, 8, 2, 3, 3, 4, 4, 4, 4]
ZERO, EPSILON, EPS_SLOPE = 1e-10, 0.005, 0.05e-6


def _around(v):
    return [v, np.nextafter(v, -np.inf), np.nextafter(v, np.inf)]


def _rand(rng, k, n, lo, hi):
    return rng.uniform(lo, hi, size=(n, k))


def grid(name, seed=7):
    rng = np.random.default_rng(seed)
    if name == "MANNING":          # Equations.hpp:54-63 (A, n, R, S)
        S = [-1.0, -1e-3, -1e-300, -0.0, 0.0, 1e-300, 1e-3, 0.5]
        rows = list(itertools.product([0.0, 1e-6, 2.5, 1e3], [0.01, 0.035, 0.2], [0.0, 1e-9, 0.3, 4.0], S))
        rnd = np.column_stack([rng.uniform(0, 50, 500), rng.uniform(0.01, 0.2, 500), rng.uniform(0, 3, 500),
                               rng.uniform(-0.05, 0.05, 500)])
    elif name == "EFFKH":          # Equations.cpp:116-134 (Ygw, aq, MacD, Kmac, AF, Kmx)
        aq, md = 30.0, 2.0
        ygw = _around(aq - md) + _around(aq) + [-1.0, 0.0, 1e-12, 5.0, 29.0, 31.0, 60.0]
        rows = list(itertools.product(ygw, [aq], [0.0, ZERO, np.nextafter(ZERO, 1), md], [0.0, 1e-4, 50.0],
                                      [0.0, 0.01, 1.0], [1e-6, 3.0]))
        rnd = np.column_stack([rng.uniform(-1, 35, 500), np.full(500, aq), rng.uniform(0, 5, 500),
                               rng.uniform(0, 100, 500), rng.uniform(0, 1, 500), rng.uniform(0, 5, 500)])
    elif name == "WEIR":           # MD_RiverFlux.cpp:65-98 (zi, yi, zj, yj, zbank, cwr, width, thr)
        zi, zb = 100.0, 100.0
        rows = []
        for yi, zj, yj, thr in itertools.product([0.0, 1e-4, 0.0002, 0.3], [97.0, 99.0, 100.0],
                                                 [0.0, 0.5, 1.0, 3.0, 5.0], _around(0.0002)):
            rows.append([zi, yi, zj, yj, zb, 0.6, 250.0, thr])
        rnd = np.column_stack([np.full(500, zi), rng.uniform(0, 0.5, 500), rng.uniform(96, 100, 500),
                               rng.uniform(0, 6, 500), np.full(500, zb), rng.uniform(0.3, 1, 500),
                               rng.uniform(10, 500, 500), np.full(500, 0.0002)])
    elif name == "R2E":            # Flux_RiverElement.cpp:11-55 (yr, zr, ye, ze, Kele, Kriv, L, D)
        rows = []
        for yr, ye, ke, kr in itertools.product([0.0, EPSILON / 2, EPSILON, 0.5, 3.0], [0.0, ZERO, 1e-9, 2.0, 27.0],
                                                [0.0, ZERO / 2, 1e-5], [0.0, 2e-5]):
            rows.append([yr, 97.0, ye, 70.0, ke, kr, 300.0, 1.5])
        for d in [ZERO, -ZERO, 0.0, 2 * ZERO, -2 * ZERO]:    # dh dead band around +-ZERO
            rows.append([1.0, 97.0, 28.0 + d, 70.0, 1e-5, 2e-5, 300.0, 1.5])
        rnd = np.column_stack([rng.uniform(0, 4, 500), np.full(500, 97.0), rng.uniform(0, 30, 500),
                               np.full(500, 70.0), rng.uniform(0, 1e-4, 500), rng.uniform(0, 1e-4, 500),
                               rng.uniform(10, 500, 500), rng.uniform(0.5, 3, 500)])
    elif name == "SATK":           # Equations.cpp:136-141 (satn, n)
        rows = list(itertools.product([ZERO * 2, 1e-6, 0.01, 0.3, 0.5, 0.9, 0.98999, 0.99], [1.05, 1.3, 1.8, 2.5, 7.0]))
        rnd = np.column_stack([rng.uniform(1e-9, 0.99, 500), rng.uniform(1.05, 6, 500)])
    elif name == "SMS":            # is_sm_et.cpp:131-140 (ThetaS, ThetaR, SatRatio)
        ths, thr = 0.45, 0.05
        b0 = thr / (ths - thr)                       # beta_s = 0 boundary
        b1 = (ths * 0.75) / (ths - thr)              # beta_s = 1 boundary
        rows = [[ths, thr, s] for s in _around(b0) + _around(b1) + [0.0, 0.2, 0.5, 1.0, 1.5]]
        rnd = np.column_stack([rng.uniform(0.3, 0.6, 500), rng.uniform(0.01, 0.1, 500), rng.uniform(0, 1, 500)])
    elif name == "DADY":           # functions.hpp:125-153 (dA, w_top, s)
        rows = list(itertools.product([-50.0, -1e-3, -0.0, 0.0, 1e-9, 2.0, 40.0], [0.0, 1e-3, 5.0, 30.0],
                                      [0.0] + _around(EPS_SLOPE) + [-EPS_SLOPE, 0.5, -0.5, 2.0]))
        rnd = np.column_stack([rng.uniform(-10, 10, 500), rng.uniform(0.1, 40, 500), rng.uniform(-2, 2, 500)])
    else:                          # River.hpp:115-127 via updateRiver (w0, bankslope, length, y)
        rows = list(itertools.product([0.0, 2.0, 25.0], [0.0, 1e-8, 0.5, 3.0], [100.0, 2500.0],
                                      [-1.0, -1e-9, 0.0, 1e-9, 0.7, 6.0]))
        rnd = np.column_stack([rng.uniform(0, 30, 500), rng.uniform(0, 3, 500), rng.uniform(50, 5000, 500),
                               rng.uniform(-0.5, 8, 500)])
    x = np.vstack([np.asarray(rows, dtype=np.float64), rnd])
    assert x.shape[1] == NIN[KAT[name]]
    return np.ascontiguousarray(x)
