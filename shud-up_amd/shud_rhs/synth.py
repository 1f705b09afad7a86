"""Synthetic SHUD meshes for the measurement configs: syn-1M / syn-10M.

Mesh: jittered structured grid (h = 100 m, node jitter U(+-0.2h)), each quad split by its Delaunay
(in-circle) diagonal; elements in row-major quad order, 2 per quad.  Surface
z = 1000 + 0.02y + 0.01|x - xbar| + 2 sin(x/700) cos(y/900), aquifer depth 30 m.  Attributes sampled from
ccw's (soil, geol, lc) rows, ccw parameter tables + calibration (packaged as data/ccw_tables.npz, made by
tests/golden/make_fixtures.py from the reference input files).  River network: main stems every M quad
columns flowing south to outlets (down = -3), tributaries in every other quad row flowing into them;
reaches of 3 quads; about 0.09 reaches and 0.5 segments per element (ccw ratios).  Derived geometry
through geometry.py (the reference's init code, restated).  Seeded, deterministic (seed 12345).
"""
import os

import numpy as np

from .geometry import river_downstream
from .model import ShudModel
from .shudio import MINRIVSLOPE, build_elements, calibrated_tables

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "ccw_tables.npz")


def load_tables():
    z = np.load(DATA, allow_pickle=False)
    cal = {str(k): float(v) for k, v in zip(z["calib_keys"], z["calib_vals"])}
    return z["soil"], z["geol"], z["lc"], z["rtype"], z["att_rows"], cal


def neighbours(tri, n_nodes):
    """nabr[j, i] = element across the edge opposite node j (Element.hpp:25), -1 on the boundary."""
    NE = tri.shape[0]
    a = np.concatenate([tri[:, 1], tri[:, 2], tri[:, 0]])
    b = np.concatenate([tri[:, 2], tri[:, 0], tri[:, 1]])
    key = np.minimum(a, b).astype(np.int64) * n_nodes + np.maximum(a, b)
    order = np.argsort(key, kind="stable")
    ks = key[order]
    same = np.nonzero(ks[1:] == ks[:-1])[0]
    e1, e2 = order[same], order[same + 1]
    nabr = np.full(3 * NE, -1, dtype=np.int64)      # slot = j*NE + i
    nabr[e1] = e2 % NE
    nabr[e2] = e1 % NE
    return nabr.reshape(3, NE)


def grid_dims(n_target):
    nqy = max(2, int(round(np.sqrt(n_target / 4.0))))
    nqx = max(2, int(round(n_target / (2.0 * nqy))))
    return nqx, nqy


def synth_model(n_target, seed=12345, h=100.0, stem_every=12, reach_quads=3):
    rng = np.random.default_rng(seed)
    soil, geol, lc, rtype, att_rows, cal = load_tables()
    nqx, nqy = grid_dims(n_target)
    nnx, nny = nqx + 1, nqy + 1
    ii, jj = np.meshgrid(np.arange(nnx), np.arange(nny))
    x = (ii * h + rng.uniform(-0.2 * h, 0.2 * h, ii.shape)).reshape(-1)
    y = (jj * h + rng.uniform(-0.2 * h, 0.2 * h, jj.shape)).reshape(-1)
    xbar = 0.5 * nqx * h
    zmax = 1000.0 + 0.02 * y + 0.01 * np.abs(x - xbar) + 2.0 * np.sin(x / 700.0) * np.cos(y / 900.0)
    aqd = np.full(x.size, 30.0)
    # quads, row-major; corners a(i,j) b(i+1,j) c(i+1,j+1) d(i,j+1)
    qi, qj = np.meshgrid(np.arange(nqx), np.arange(nqy))
    qi, qj = qi.reshape(-1), qj.reshape(-1)
    A = qj * nnx + qi
    B = A + 1
    Cn = A + nnx + 1
    D = A + nnx
    # in-circle test of d against (a, b, c) (a,b,c anticlockwise): d inside -> use diagonal b-d
    ax, ay, bx, by, cx, cy, dx, dy = x[A], y[A], x[B], y[B], x[Cn], y[Cn], x[D], y[D]
    adx, ady, bdx, bdy, cdx, cdy = ax - dx, ay - dy, bx - dx, by - dy, cx - dx, cy - dy
    det = ((adx * adx + ady * ady) * (bdx * cdy - cdx * bdy) - (bdx * bdx + bdy * bdy) * (adx * cdy - cdx * ady)
           + (cdx * cdx + cdy * cdy) * (adx * bdy - bdx * ady))
    use_bd = det > 0
    t0 = np.where(use_bd[:, None], np.stack([A, B, D], 1), np.stack([A, B, Cn], 1))
    t1 = np.where(use_bd[:, None], np.stack([B, Cn, D], 1), np.stack([A, Cn, D], 1))
    tri = np.empty((2 * qi.size, 3), dtype=np.int64)
    tri[0::2] = t0
    tri[1::2] = t1
    NE = tri.shape[0]
    nabr = neighbours(tri, x.size)
    # attributes: ccw (soil, geol, lc) rows
    pick = att_rows[rng.integers(0, att_rows.shape[0], NE)]
    S, G, L, R, g = calibrated_tables(soil, geol, lc, rtype, cal)

    # ---------------- river network ----------------
    M = stem_every
    stems = np.arange(M // 2, nqx, M)
    reach_cells = []        # list of (quad cells list [(i,j)...] upstream->downstream, type)
    down_of = []            # filled after ids are known
    # stems: reaches of `reach_quads` rows, flowing south; reach r covers rows [j0, j0+rq)
    stem_reach = {}         # (stem idx, row) -> reach id
    reaches = []            # (kind, key, cells, type)
    for j0 in range(0, nqy, reach_quads):
        for k, c in enumerate(stems):
            rows = list(range(min(nqy, j0 + reach_quads) - 1, j0 - 1, -1))   # upstream (north) first
            reaches.append(("stem", (k, j0), [(c, r) for r in rows], 4))
        if True:
            for jr in range(j0, min(nqy, j0 + reach_quads)):
                if jr % 2:
                    continue
                for k, c in enumerate(stems):
                    lo, hi = c - M // 2 + 1, c - 1             # west tributary cols [lo, hi], flows east
                    west = list(range(max(0, lo), hi + 1))
                    ro, rh = c + 1, min(nqx - 1, c + M - M // 2 - 1)  # east tributary, flows west
                    east = list(range(rh, ro - 1, -1))
                    for side, cols in (("w", west), ("e", east)):
                        for q in range(0, len(cols), reach_quads):
                            part = cols[q:q + reach_quads]
                            reaches.append(("trib", (k, jr, side, q), [(ci, jr) for ci in part], 1 + (q // reach_quads) % 3))
    NR = len(reaches)
    rid = {(kind, key): n for n, (kind, key, _, _) in enumerate(reaches)}
    down = np.empty(NR, dtype=np.int64)
    rtyp = np.empty(NR, dtype=np.int64)
    for n, (kind, key, cells, ty) in enumerate(reaches):
        rtyp[n] = ty
        if kind == "stem":
            k, j0 = key
            down[n] = rid[("stem", (k, j0 - reach_quads))] if j0 - reach_quads >= 0 else -3
        else:
            k, jr, side, q = key
            nxt = ("trib", (k, jr, side, q + reach_quads))
            if nxt in rid:
                down[n] = rid[nxt]
            else:
                down[n] = rid[("stem", (k, (jr // reach_quads) * reach_quads))]
    # segments: 2 per quad cell (both triangles), ordered by reach (rivseg is sorted by iRiv)
    seg_ele, seg_riv, seg_len = [], [], []
    for n, (kind, key, cells, ty) in enumerate(reaches):
        for (ci, cj) in cells:
            e0 = 2 * (cj * nqx + ci)
            seg_ele += [e0, e0 + 1]
            seg_riv += [n, n]
    seg_ele = np.array(seg_ele, dtype=np.int64)
    seg_riv = np.array(seg_riv, dtype=np.int64)
    NS = seg_ele.size
    seg_len = 0.5 * h * (1.0 + rng.uniform(-0.2, 0.2, NS))
    riv_id = np.zeros(NE, dtype=np.int64)
    riv_id[seg_ele] = seg_riv + 1

    ele, par, ext = build_elements(tri, nabr, x, y, zmax, aqd, pick[:, 0], pick[:, 1], pick[:, 2], S, G, L,
                                   riv_id, g["AQ_DEPTH+"])
    length = np.bincount(seg_riv, weights=seg_len, minlength=NR)
    # bed slope from the surface drop between the first and last element of the reach
    first = np.zeros(NR, dtype=np.int64)
    last = np.zeros(NR, dtype=np.int64)
    first[seg_riv[::-1]] = seg_ele[::-1]
    last[seg_riv] = seg_ele
    zs = ele["z_surf"]
    slope = np.abs(zs[first] - zs[last]) / length
    slope = np.where(MINRIVSLOPE < slope, slope, MINRIVSLOPE)
    rt = rtyp - 1
    rrough = R["rivRough"][rt]
    avg_r, d2d = river_downstream(down, length, rrough)
    m = ShudModel(NE, NR, NS, 1)
    m.ele = ele
    m.nabr = nabr.reshape(-1)
    m.ibc = np.zeros(NE, dtype=np.int32)
    m.iss = np.zeros(NE, dtype=np.int32)
    m.par = par
    m.riv = dict(riv_length=length, riv_bed_slope=slope, riv_dist2down=d2d, riv_avg_rough=avg_r,
                 riv_depth=R["depth"][rt], riv_bottom_width=R["BottomWidth"][rt], riv_bankslope=R["bankslope"][rt],
                 riv_ksath=R["KsatH"][rt], riv_bedthick=R["BedThick"][rt])
    m.riv_down = down.astype(np.int32)
    m.riv_bc = np.zeros(NR, dtype=np.int32)
    m.seg_ele = seg_ele.astype(np.int32)
    m.seg_riv = seg_riv.astype(np.int32)
    m.seg_length = seg_len
    m.seg_cwr = R["Cwr"][rt[seg_riv]]
    m.meta.update(prj=f"syn-{NE}", nqx=nqx, nqy=nqy, x=ext["x"], y=ext["y"], seed=seed)
    return m.finalize()
