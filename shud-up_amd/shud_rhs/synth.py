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


def _down_key(kind, key, rid, reach_quads):
    """the downstream reach's (kind, key) of a reach, or None at an outlet (synth_model's network rule)"""
    if kind == "stem":
        k, j0 = key
        return ("stem", (k, j0 - reach_quads)) if j0 - reach_quads >= 0 else None
    k, jr, side, q = key
    nxt = ("trib", (k, jr, side, q + reach_quads))
    return nxt if nxt in rid else ("stem", (k, (jr // reach_quads) * reach_quads))


def _tree_reach_order(reaches, reach_quads, depth_first=False):
    """The reaches renumbered from the outlets, breadth-first (each reach's upstream reaches, in their generated
    order, numbered consecutively and next to the upstream reaches of the reach numbered before it) or
    depth-first pre-order (a reach's first upstream reach numbered right after it).  A caller
    numbering for the river-order measurement: same network, same cells, other reach ids."""
    rid = {(kind, key): n for n, (kind, key, _, _) in enumerate(reaches)}
    ups = [[] for _ in reaches]
    outlets = []
    for n, (kind, key, _, _) in enumerate(reaches):
        dk = _down_key(kind, key, rid, reach_quads)
        (outlets if dk is None else ups[rid[dk]]).append(n)
    if not depth_first:
        order, head = list(outlets), 0
        while head < len(order):
            order.extend(ups[order[head]])
            head += 1
    else:   # pre-order: a reach, then each upstream subtree in turn (a chain of single reaches stays contiguous)
        order, stack = [], list(reversed(outlets))
        while stack:
            n = stack.pop()
            order.append(n)
            stack.extend(reversed(ups[n]))
    assert len(order) == len(reaches)
    return [reaches[n] for n in order]


def synth_model(n_target, seed=12345, h=100.0, stem_every=12, reach_quads=3, reach_order="band"):
    """reach_order: "band" (the generated order: row bands south to north, stems then tributaries) or "bfs"
    / "dfs" (_tree_reach_order; the segment lengths' random draws then land on other segments)."""
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
    if reach_order in ("bfs", "dfs"):
        reaches = _tree_reach_order(reaches, reach_quads, depth_first=reach_order == "dfs")
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


# ---------------------------------------------------------------------------------------------------------
# SHUD text-format project writer ("the synthetic-mesh generator at scale"): the same seeded
# mesh / river tree as synth_model, written as the reference's input files so the C++ host (shud_gpu,
# include/shud_host.h) and the Python readers (shudio) can load it like input/<prj>/.  Numbers are written
# with 17 significant digits, so every value reads back bit for bit.
# ---------------------------------------------------------------------------------------------------------
def _fmt(v):
    return f"{float(v):.17g}" if isinstance(v, (float, np.floating)) else str(int(v))


def _write_table(f, header, rows, extra=""):
    rows = list(rows)
    ncol = len(header)
    f.write(f"{len(rows)}\t{ncol}{extra}\n")
    f.write("\t".join(header) + "\n")
    for r in rows:
        f.write("\t".join(_fmt(v) for v in r) + "\n")


def synth_raw(n_target, seed=12345, h=100.0, stem_every=12, reach_quads=3):
    """Raw (file-level) description of synth_model's mesh: nodes, triangles, neighbours, attribute rows,
    reaches and segments, with the random draws in synth_model's order."""
    m = synth_model(n_target, seed=seed, h=h, stem_every=stem_every, reach_quads=reach_quads)
    rng = np.random.default_rng(seed)
    soil, geol, lc, rtype, att_rows, cal = load_tables()
    nqx, nqy = grid_dims(n_target)
    nnx, nny = nqx + 1, nqy + 1
    ii, jj = np.meshgrid(np.arange(nnx), np.arange(nny))
    x = (ii * h + rng.uniform(-0.2 * h, 0.2 * h, ii.shape)).reshape(-1)
    y = (jj * h + rng.uniform(-0.2 * h, 0.2 * h, jj.shape)).reshape(-1)
    xbar = 0.5 * nqx * h
    zmax = 1000.0 + 0.02 * y + 0.01 * np.abs(x - xbar) + 2.0 * np.sin(x / 700.0) * np.cos(y / 900.0)
    qi, qj = np.meshgrid(np.arange(nqx), np.arange(nqy))
    qi, qj = qi.reshape(-1), qj.reshape(-1)
    A = qj * nnx + qi
    B, Cn, D = A + 1, A + nnx + 1, A + nnx
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
    pick = att_rows[rng.integers(0, att_rows.shape[0], tri.shape[0])]
    return m, dict(x=x, y=y, zmax=zmax, aqd=np.full(x.size, 30.0), tri=tri, pick=pick, soil=soil, geol=geol,
                   lc=lc, rtype=rtype, cal=cal)


def write_project(outdir, prj, n_target, days=2.0, seed=12345, max_step=10.0, et_step=60.0, dt_out=60,
                  forcing_dt_min=60.0, extra_para=None, bc=False, cfg_output=False, lake=False):
    """Write input files <outdir>/<prj>.* for the synthetic mesh; returns the in-memory ShudModel.
    bc: a few elements / reaches get boundary conditions (iBC = +-1, +-2; BC = +-1) with hourly .tsd.ebc1/.ebc2/
    .rbc1/.rbc2 tables.  cfg_output: a .cfg.output switching some element / reach columns off.
    lake: one lake (iLake = 1, MD_readin.cpp:262-263) over a 10 x 10-quad patch of the mesh, with a three-row
    <prj>.lake.bathy (MD_Lake.cpp:147-168) and its stage as the cfg.ic's third table."""
    os.makedirs(outdir, exist_ok=True)
    m, raw = synth_raw(n_target, seed=seed)
    NE, NR, NS = m.num_ele, m.num_riv, m.num_seg
    ibc = np.zeros(NE, dtype=np.int64)
    rbc = np.zeros(NR, dtype=np.int64)
    if bc:
        rng_bc = np.random.default_rng(seed + 7)
        riv_ele = np.zeros(NE, dtype=bool)
        riv_ele[m.seg_ele] = True
        cand = np.nonzero(~riv_ele)[0]
        pick_e = rng_bc.choice(cand, 8, replace=False)
        ibc[pick_e] = [1, 2, 1, 2, -1, -2, -1, -2]
        pick_r = rng_bc.choice(NR, 4, replace=False)
        rbc[pick_r] = [1, -1, 1, -1]
    ilake = np.zeros(NE, dtype=np.int64)
    if lake:
        nqx, nqy = grid_dims(n_target)
        qi0, qj0 = nqx // 3, nqy // 3
        qs = [(qj0 + b) * nqx + qi0 + a for b in range(10) for a in range(10)]
        ilake[np.array([2 * q + t for q in qs for t in (0, 1)])] = 1
    p = lambda ext: os.path.join(outdir, f"{prj}.{ext}")
    nbr = m.nabr.reshape(3, NE)
    with open(p("sp.mesh"), "w") as f:
        _write_table(f, ["ID", "Node1", "Node2", "Node3", "Nabr1", "Nabr2", "Nabr3", "Zmax"],
                     ([i + 1, *(raw["tri"][i] + 1), *(nbr[:, i] + 1), 0] for i in range(NE)))
        _write_table(f, ["ID", "X", "Y", "AqDepth", "Elevation"],
                     ([k + 1, raw["x"][k], raw["y"][k], raw["aqd"][k], raw["zmax"][k]] for k in range(raw["x"].size)))
    pick = raw["pick"]
    with open(p("sp.att"), "w") as f:
        _write_table(f, ["INDEX", "SOIL", "GEOL", "LC", "FORC", "MF", "BC", "SS", "LAKE"],
                     ([i + 1, pick[i, 0], pick[i, 1], pick[i, 2], 1, 1, ibc[i], 0, ilake[i]] for i in range(NE)))
    if lake:
        zl = float(np.min(m.ele["z_surf"][ilake > 0])) - 3.0
        with open(p("lake.bathy"), "w") as f:
            _write_table(f, ["Index", "Y", "Area"], [[1, zl, 2.0e4], [2, zl + 5.0, 1.5e5], [3, zl + 20.0, 4.0e5]])
    for ext, tab in (("para.soil", raw["soil"]), ("para.geol", raw["geol"]), ("para.lc", raw["lc"])):
        with open(p(ext), "w") as f:
            _write_table(f, [f"C{j}" for j in range(tab.shape[1])], ([int(r[0])] + [float(v) for v in r[1:]] for r in tab))
    # reaches: type recovered from the parameter rows (riv_depth identifies the rtype row uniquely)
    R = raw["rtype"]
    cal = dict(raw["cal"])
    depth_rows = R[:, 1] + cal.get("RIV_DPTH+", 1.0)
    rt = np.array([int(np.nonzero(depth_rows == d)[0][0]) for d in m.riv["riv_depth"]])
    down = m.riv_down.astype(np.int64)
    with open(p("sp.riv"), "w") as f:
        _write_table(f, ["Index", "Down", "Type", "Slope", "Length", "BC"],
                     ([r + 1, down[r] + 1 if down[r] >= 0 else down[r], rt[r] + 1, float(m.riv["riv_bed_slope"][r]),
                       float(m.riv["riv_length"][r]), rbc[r]] for r in range(NR)))
        _write_table(f, ["Index", "Depth", "BankSlope", "Width", "Sinuosity", "Manning", "Cwr", "KsatH", "BedThick"],
                     ([int(r[0])] + [float(v) for v in r[1:]] for r in R))
    with open(p("sp.rivseg"), "w") as f:
        _write_table(f, ["Index", "iRiv", "iEle", "Length"],
                     ([s + 1, int(m.seg_riv[s]) + 1, int(m.seg_ele[s]) + 1, float(m.seg_length[s])] for s in range(NS)))
    with open(p("cfg.calib"), "w") as f:
        for k, v in sorted(cal.items()):
            f.write(f"{k}\t{float(v):.17g}\n")
    para = {"INIT_MODE": 3, "ABSTOL": 1e-4, "RELTOL": 1e-4, "INIT_SOLVER_STEP": 1, "MAX_SOLVER_STEP": max_step,
            "LSM_STEP": et_step, "START": 0, "END": days, "TERRAIN_RADIATION": 1, "dt_ye_surf": dt_out,
            "dt_ye_unsat": dt_out, "dt_ye_gw": dt_out, "dt_ye_snow": dt_out, "dt_qe_et": dt_out,
            "dt_qe_prcp": dt_out, "dt_qe_infil": dt_out, "dt_qe_rech": dt_out, "dt_Qe_sub": dt_out,
            "dt_Qe_surf": dt_out, "dt_yr_stage": dt_out, "dt_Qr_down": dt_out, "dt_Qr_up": dt_out,
            "dt_Qr_surf": dt_out, "dt_Qr_sub": dt_out}
    para.update(extra_para or {})
    with open(p("cfg.para"), "w") as f:
        for k, v in para.items():
            f.write(f"{k}\t{v}\n")
    # initial condition (INIT_MODE 3): wet surface in the valleys, unsat 20 %, gw 60 % of the aquifer
    rng = np.random.default_rng(seed + 1)
    aq = m.par["aquifer_depth"]
    with open(p("cfg.ic"), "w") as f:
        _write_table(f, ["Index", "Canopy", "Snow", "Surface", "Unsat", "GW"],
                     ([i + 1, 0.0, 0.0, float(rng.uniform(0, 0.01)), float(0.2 * aq[i]), float(0.6 * aq[i])]
                      for i in range(NE)))
        _write_table(f, ["Index", "Stage"], ([r + 1, float(rng.uniform(0.1, 1.0))] for r in range(NR)))
        if lake:
            _write_table(f, ["Index", "Stage"], [[1, 3.5]])
    # forcing: one station (ccw's coordinates), hourly prcp/temp/rh/wind/radiation, 20000101
    nrow = int(np.ceil(days * 1440.0 / forcing_dt_min)) + 2
    tday = np.arange(nrow) * forcing_dt_min / 1440.0
    hour = (tday * 24.0) % 24.0
    temp = 8.0 + 6.0 * np.sin((hour - 9.0) / 24.0 * 2 * np.pi) + rng.normal(0, 0.5, nrow)
    prcp = np.where(rng.uniform(0, 1, nrow) < 0.15, rng.gamma(1.5, 8.0, nrow), 0.0)
    rh = np.clip(0.6 + 0.2 * np.cos(hour / 24.0 * 2 * np.pi) + rng.normal(0, 0.05, nrow), 0.05, 1.0)
    wind = np.abs(2.0 + rng.normal(0, 0.8, nrow))
    rad = np.maximum(0.0, 800.0 * np.sin((hour - 6.0) / 12.0 * np.pi)) * (hour > 6) * (hour < 18)
    with open(os.path.join(outdir, "forcing.csv"), "w") as f:
        f.write(f"{nrow}\t6\t20000101\t20100101\n")
        f.write("Time_Day\tAPCP\tTMP\tSPFH\tUGRD\tDSWRF\n")
        for k in range(nrow):
            f.write(f"{tday[k]:.17g}\t{prcp[k]:.17g}\t{temp[k]:.17g}\t{rh[k]:.17g}\t{wind[k]:.17g}\t{rad[k]:.17g}\n")
    with open(p("tsd.forc"), "w") as f:
        f.write("1 20000101\n\nID\tLon\tLat\tX\tY\tZ\tFilename\n")
        f.write("1\t-122.71\t39.195\t0\t0\t-9999\tforcing.csv\n")
    if bc:
        # hourly BC tables: element heads (ebc1, m), element fluxes (ebc2, m3/min), river stages / fluxes
        nh = int(np.ceil(days * 24)) + 2
        aqm = float(np.median(m.par["aquifer_depth"]))
        tabs = {"tsd.ebc1": [0.5 * aqm + 0.1 * np.sin(np.arange(nh) / 5.0), 0.7 * aqm + 0.05 * np.cos(np.arange(nh) / 7.0)],
                "tsd.ebc2": [-0.02 + 0.01 * np.sin(np.arange(nh) / 3.0), 0.03 + 0.0 * np.arange(nh)],
                "tsd.rbc1": [0.8 + 0.2 * np.sin(np.arange(nh) / 4.0)],
                "tsd.rbc2": [5.0 + 2.0 * np.cos(np.arange(nh) / 6.0)]}
        for ext, cols in tabs.items():
            with open(p(ext), "w") as f:
                f.write(f"{nh}\t{len(cols) + 1}\t20000101\n")
                f.write("Time_Day\t" + "\t".join(f"X{j + 1}" for j in range(len(cols))) + "\n")
                for k in range(nh):
                    f.write(f"{k / 24.0:.17g}\t" + "\t".join(f"{c[k]:.17g}" for c in cols) + "\n")
    if cfg_output:
        with open(p("cfg.output"), "w") as f:
            # element table: header default 1 (atoi of "1 ..."), a few columns off; river table: default 0
            off = np.arange(0, NE, max(1, NE // 7))
            _write_table(f, ["1", "ON"], ([int(i) + 1, 0] for i in off))
            on = np.arange(0, NR, max(1, NR // 5))
            f.write(f"{len(on)}\t2\n0\tON\n")
            for r in on:
                f.write(f"{int(r) + 1}\t1\n")
    nlc = raw["lc"].shape[0]
    months = int(days // 31) + 3
    with open(p("tsd.lai"), "w") as f:
        f.write(f"{months}\t{nlc + 1}\t20000101\n")
        f.write("Time_Day\t" + "\t".join(f"X{j + 1}" for j in range(nlc)) + "\n")
        for k in range(months):
            f.write(f"{31 * k}\t" + "\t".join(f"{0.5 + 0.1 * j + 0.05 * k:.17g}" for j in range(nlc)) + "\n")
    with open(p("tsd.mf"), "w") as f:
        f.write(f"{months}\t2\t20000101\n")
        f.write("Time_Day\tMF\n")
        for k in range(months):
            f.write(f"{31 * k}\t{0.0013 + 0.0001 * k:.17g}\n")
    return m
