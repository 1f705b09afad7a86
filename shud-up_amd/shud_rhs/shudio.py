"""SHUD text-input reader + Model_Data initialisation (host side, numpy), restating the reference.

Readers:  TabularData::read (src/classes/TabularData.cpp:27-55: "nrow ncol" line, header line, rows
parsed with strtold then stored as double), Model_Data::read_mesh/att/soil/geol/lc/riv/rivseg
(src/ModelData/MD_readin.cpp:106-363), globalCal::read/push (src/classes/ModelConfigure.cpp:140-260,
443-459), Control_Data `.cfg.para` keys CLOSEBOUNDARY (src/classes/Model_Control.cpp:175-176).
Init:  Model_Data::initialize (src/ModelData/MD_initialize.cpp:168-245) via geometry.py, calibration
(ModelConfigure.cpp:79-139, River.cpp:36-45), LoadIC mode 3 (MD_initialize.cpp:66-108).

Lakes: lake ids from the .sp.att LAKE column, bathymetry tables from .lake.bathy
(Model_Data::lake_readBathy, MD_Lake.cpp:147-168: one TabularData block per lake, columns INDEX, yi, ai),
lake stages from the third .cfg.ic table (MD_initialize.cpp:86-99; 2.0 when the row count mismatches).
"""
import os

import numpy as np

from .geometry import (apply_nabor, element_geometry, node_zmin, river_downstream, rm_sinks)
from .model import ShudModel

MINRIVSLOPE = 4e-4                 # Macros.hpp:47
FieldCapacityRatio = 0.75


def _num(tok):
    # (double) strtold(tok): parse in long double then round once to double
    return float(np.longdouble(tok))


def read_table(path_or_lines, start=0):
    """TabularData::read -> (array [nrow, ncol] float64, next line index)."""
    lines = path_or_lines
    if isinstance(path_or_lines, str):
        with open(path_or_lines) as f:
            lines = f.read().splitlines()
    dims = lines[start].split()
    nrow, ncol = int(dims[0]), int(dims[1])
    out = np.zeros((nrow, ncol))
    for r in range(nrow):
        toks = lines[start + 2 + r].split()
        for c in range(min(ncol, len(toks))):
            try:
                out[r, c] = _num(toks[c])
            except ValueError:
                out[r, c] = 0.0
    return out, start + 2 + nrow


def read_keyvals(path):
    d = {}
    with open(path) as f:
        for line in f:
            if not line or line[0] in "#\n \0":
                continue
            t = line.split()
            if len(t) >= 2:
                try:
                    d[t[0].upper()] = float(t[1])
                except ValueError:
                    pass
    return d


# calibration defaults: calib_* classes (ModelConfigure.hpp:12-41, River.hpp:15-25)
CALIB_DEFAULTS = {
    "GEOL_KSATH": 1.0, "GEOL_KSATV": 1.0, "GEOL_KMACSATH": 1.0, "GEOL_DMAC": 1.0, "GEOL_THETAS": 1.0,
    "GEOL_THETAR": 1.0, "GEOL_MACVF": 1.0,
    "SOIL_KINF": 1.0, "SOIL_KMACSATV": 1.0, "SOIL_DINF": 1.0, "SOIL_ALPHA": 1.0, "SOIL_BETA": 1.0,
    "SOIL_MACHF": 1.0,
    "LC_VEGFRAC": 1.0, "LC_ALBEDO": 1.0, "LC_ROUGH": 1.0, "LC_SOILDGD": 1.0, "LC_DROOT": 1.0, "LC_IMPAF": 1.0,
    "AQ_DEPTH+": 0.0,
    "RIV_ROUGH": 1.0, "RIV_KH": 1.0, "RIV_CWR": 1.0, "RIV_DPTH+": 1.0, "RIV_WDTH+": 1.0, "RIV_BSLOPE+": 1.0,
    "RIV_SINU": 1.0, "RIV_BEDTHICK": 1.0,
}


def calibrated_tables(soil, geol, lc, rtype, cal):
    """Soil/Geol/Landcover/river_para applyCalib (ModelConfigure.cpp:79-139, River.cpp:23-45)."""
    g = dict(CALIB_DEFAULTS)
    g.update(cal)
    S = {}
    S["infKsatV"] = soil[:, 1] / 1440.0 * g["SOIL_KINF"]
    S["ThetaS"] = soil[:, 2].copy()
    S["ThetaR"] = soil[:, 3].copy()
    S["infD"] = soil[:, 4] * g["SOIL_DINF"]
    S["Alpha"] = soil[:, 5] * g["SOIL_ALPHA"]
    beta = soil[:, 6] * g["SOIL_BETA"]
    S["Beta"] = np.where(beta < 1.1, 1.1, beta)
    S["hAreaF"] = soil[:, 7] * g["SOIL_MACHF"]
    S["macKsatV"] = soil[:, 8] / 1440.0 * g["SOIL_KMACSATV"]
    G = {}
    G["KsatH"] = geol[:, 1] / 1440.0 * g["GEOL_KSATH"]
    G["KsatV"] = geol[:, 2] / 1440.0 * g["GEOL_KSATV"]
    G["geo_ThetaS"] = geol[:, 3].copy()
    G["geo_ThetaR"] = geol[:, 4].copy()
    G["geo_vAreaF"] = geol[:, 5] * g["GEOL_MACVF"]
    G["macKsatH"] = geol[:, 6] / 1440.0 * g["GEOL_KMACSATH"]
    G["macD"] = geol[:, 7] * g["GEOL_DMAC"]
    G["Sy"] = g["GEOL_THETAS"] * G["geo_ThetaS"] - g["GEOL_THETAR"] * G["geo_ThetaR"]
    L = {}
    L["Albedo"] = lc[:, 1] * g["LC_ALBEDO"]
    L["VegFrac"] = lc[:, 2] * g["LC_VEGFRAC"]
    L["Rough"] = lc[:, 3] / 60.0 * g["LC_ROUGH"]
    L["RzD"] = lc[:, 4] * g["LC_DROOT"]
    L["SoilDgrd"] = lc[:, 5] * g["LC_SOILDGD"]
    L["ImpAF"] = lc[:, 6] * g["LC_IMPAF"]
    R = {}
    if rtype is not None and len(rtype):
        R["depth"] = rtype[:, 1] + g["RIV_DPTH+"]
        R["bankslope"] = rtype[:, 2] + g["RIV_BSLOPE+"]
        R["BottomWidth"] = rtype[:, 3] + g["RIV_WDTH+"]
        R["rivRough"] = rtype[:, 5] / 60.0 * g["RIV_ROUGH"]
        R["Cwr"] = rtype[:, 6] * g["RIV_CWR"]
        R["KsatH"] = rtype[:, 7] / 1440.0 * g["RIV_KH"]
        R["BedThick"] = rtype[:, 8] * g["RIV_BEDTHICK"]
    return S, G, L, R, g


def build_elements(tri, nabr, nodes_x, nodes_y, nodes_zmax, nodes_aqd, isoil, igeol, ilc, S, G, L,
                   riv_id, c_aqd=0.0):
    """MD_initialize.cpp:173-197: geometry, copyGeol/Soil/Landc, InitElement, SoilDgrd/ImpAF
    multipliers, rmSinks (+ its InitElement), applyNabor.  Returns (ele dict, par dict, extras)."""
    zmin = node_zmin(nodes_zmax, nodes_aqd, c_aqd)
    geo = element_geometry(nodes_x, nodes_y, nodes_zmax, zmin, tri)
    s, gi, l = isoil - 1, igeol - 1, ilc - 1
    par = {}
    par["KsatH"] = G["KsatH"][gi]; par["KsatV"] = G["KsatV"][gi]; par["geo_vAreaF"] = G["geo_vAreaF"][gi]
    par["macKsatH"] = G["macKsatH"][gi]; macD = G["macD"][gi].copy(); par["Sy"] = G["Sy"][gi]
    par["infKsatV"] = S["infKsatV"][s].copy(); par["ThetaS"] = S["ThetaS"][s]; par["ThetaR"] = S["ThetaR"][s]
    par["Beta"] = S["Beta"][s]; par["hAreaF"] = S["hAreaF"][s]; par["macKsatV"] = S["macKsatV"][s].copy()
    par["infD"] = S["infD"][s]
    vegfrac = L["VegFrac"][l].copy(); rough = L["Rough"][l]; par["RzD"] = L["RzD"][l]
    soildgrd = L["SoilDgrd"][l]; par["ImpAF"] = L["ImpAF"][l]
    # InitElement (Element.cpp:218-237), first call
    aq = geo["z_surf"] - geo["z_bottom"]
    macD = np.where(aq < macD, aq, macD)
    par["infKsatV"] = par["infKsatV"] * (1 - soildgrd)
    par["macKsatV"] = par["macKsatV"] * (1 - soildgrd)
    par["VegFrac"] = vegfrac * (1 - par["ImpAF"])
    z_surf, z_bottom, raised = rm_sinks(geo["z_surf"], geo["z_bottom"], aq, nabr, riv_id)
    aq = z_surf - z_bottom                          # InitElement inside rmSinks
    macD = np.where(aq < macD, aq, macD)
    par["aquifer_depth"] = aq
    par["macD"] = macD
    d2n, avg = apply_nabor(nabr, geo["x"], geo["y"], rough, geo["dist2edge"])
    ele = dict(area=geo["area"], z_surf=z_surf, z_bottom=z_bottom, depression=np.full(aq.size, 0.0002),
               rough=rough, edge=geo["edge"].reshape(-1), dist2nabor=d2n.reshape(-1),
               dist2edge=geo["dist2edge"].reshape(-1), avg_rough=avg.reshape(-1))
    return ele, {k: np.ascontiguousarray(v, dtype=np.float64) for k, v in par.items()}, \
        dict(x=geo["x"], y=geo["y"], raised=raised)


def load_project(indir, prj, end_override=None):
    """Read input/<prj>/ and return (ShudModel, extras).  extras holds the IC state y0."""
    p = lambda ext: os.path.join(indir, f"{prj}.{ext}")
    with open(p("sp.mesh")) as f:
        lines = f.read().splitlines()
    mesh, nxt = read_table(lines, 0)
    nodes, _ = read_table(lines, nxt)
    NE = mesh.shape[0]
    tri = mesh[:, 1:4].astype(np.int64) - 1
    nabr = (mesh[:, 4:7].astype(np.int64) - 1).T.copy()          # [3, NE], file 0 -> -1 boundary
    nabr = np.where(nabr < -1, -1, nabr)                          # (negative = lake neighbour: out of scope)
    # Node[node[k] - 1]: positional rows (Element.cpp:68-79), the index column is not consulted
    att, _ = read_table(p("sp.att"))
    soil, _ = read_table(p("para.soil"))
    geol, _ = read_table(p("para.geol"))
    lc, _ = read_table(p("para.lc"))
    with open(p("sp.riv")) as f:
        rl = f.read().splitlines()
    riv, nxt = read_table(rl, 0)
    rtype, _ = read_table(rl, nxt)
    rivseg, _ = read_table(p("sp.rivseg"))
    cal = read_keyvals(p("cfg.calib"))
    para = read_keyvals(p("cfg.para"))
    close_boundary = int(para.get("CLOSEBOUNDARY", 1))
    S, G, L, R, g = calibrated_tables(soil, geol, lc, rtype, cal)
    NR, NS = riv.shape[0], rivseg.shape[0]
    seg_riv = rivseg[:, 1].astype(np.int64) - 1
    seg_ele = rivseg[:, 2].astype(np.int64) - 1
    riv_id = np.zeros(NE, dtype=np.int64)
    riv_id[seg_ele] = seg_riv + 1                                 # MD_initialize.cpp:188-191
    ele, par, ext = build_elements(tri, nabr, nodes[:, 1], nodes[:, 2], nodes[:, 4], nodes[:, 3],
                                   att[:, 1].astype(np.int64), att[:, 2].astype(np.int64),
                                   att[:, 3].astype(np.int64), S, G, L, riv_id, g["AQ_DEPTH+"])
    m = ShudModel(NE, NR, NS, close_boundary)
    m.ele = ele
    m.nabr = nabr.reshape(-1)
    m.ibc = att[:, 6].astype(np.int32)
    m.iss = att[:, 7].astype(np.int32)
    m.ilake = att[:, 8].astype(np.int32)
    m.par = par
    # rivers: initialRiver/applyParameter (River.cpp:63-94), BedSlope >= MINRIVSLOPE (MD_initialize.cpp:211-215)
    rdown = riv[:, 1].astype(np.int64)
    rt = riv[:, 2].astype(np.int64) - 1
    length = riv[:, 4].copy()
    bedslope = np.where(MINRIVSLOPE < riv[:, 3], riv[:, 3], MINRIVSLOPE)   # max(a,b) = a < b ? b : a
    down0 = np.where(rdown > 0, rdown - 1, rdown)                  # 0-based, negative outlet codes kept
    if np.any(rdown == 0):
        raise ValueError("river reach with down == 0: reference exits (MD_RiverFlux.cpp:55-57)")
    rrough = R["rivRough"][rt]
    avg_r, d2d = river_downstream(down0, length, rrough)
    m.riv = dict(riv_length=length, riv_bed_slope=bedslope, riv_dist2down=d2d, riv_avg_rough=avg_r,
                 riv_depth=R["depth"][rt], riv_bottom_width=R["BottomWidth"][rt], riv_bankslope=R["bankslope"][rt],
                 riv_ksath=R["KsatH"][rt], riv_bedthick=R["BedThick"][rt])
    m.riv_down = down0.astype(np.int32)
    m.riv_bc = riv[:, 5].astype(np.int32)
    m.seg_ele = seg_ele.astype(np.int32)
    m.seg_riv = seg_riv.astype(np.int32)
    m.seg_length = rivseg[:, 3].copy()
    m.seg_cwr = R["Cwr"][rt[seg_riv]]                              # MD_initialize.cpp:220-226
    # lakes: lakeon when any iLake > 0 (MD_readin.cpp:262-263); NumLake = LakeUniqueID (MD_Lake.cpp:12-29)
    if np.any(m.ilake > 0):
        NL = int(np.unique(m.ilake[m.ilake > 0]).size)
        with open(p("lake.bathy")) as f:
            bl = f.read().splitlines()
        off, ys, as_, nxt = [0], [], [], 0
        for _ in range(NL):
            tb, nxt = read_table(bl, nxt)
            ys.append(tb[:, 1])
            as_.append(tb[:, 2])
            off.append(off[-1] + tb.shape[0])
        m.num_lake = NL
        m.lake_bathy_off = np.array(off, dtype=np.int32)
        m.lake_bathy_y = np.concatenate(ys)
        m.lake_bathy_a = np.concatenate(as_)
    m.finalize()
    # IC (INIT_MODE 3): .cfg.ic element table [idx, canopy, snow, surf, unsat, gw], then river stage
    y0 = None
    if os.path.exists(p("cfg.ic")):
        with open(p("cfg.ic")) as f:
            il = f.read().splitlines()
        ice, nxt = read_table(il, 0)
        icr, nxt = read_table(il, nxt)
        parts = [ice[:NE, 3], ice[:NE, 4], ice[:NE, 5], icr[:NR, 1]]
        if m.num_lake:
            icl, _ = read_table(il, nxt)
            parts.append(icl[:, 1] if icl.shape[0] == m.num_lake else np.full(m.num_lake, 2.))
        y0 = np.concatenate(parts)
    m.meta.update(prj=prj, x=ext["x"], y=ext["y"], raised=ext["raised"], close_boundary=close_boundary)
    return m, {"y0": y0, "S": S, "G": G, "L": L, "R": R, "calib": g, "att": att}


def read_dat(path):
    """Read a SHUD binary output file as Print_Ctrl writes it (src/classes/Model_Control.cpp:727-735, 893-899):
    a 1024-byte text header, StartTime and NumVar as doubles, icol[NumVar] (1-based column ids as doubles),
    then rows of (t, value[NumVar]) doubles, t = left endpoint of the output interval [min]."""
    raw = np.fromfile(path, dtype=np.uint8)
    header = raw[:1024].tobytes().split(b"\0", 1)[0].decode()
    body = raw[1024:].view(np.float64)
    start_time, nvar = body[0], int(body[1])
    icol = body[2:2 + nvar].astype(np.int64)
    rows = body[2 + nvar:]
    if rows.size % (nvar + 1):
        raise ValueError(f"{path}: {rows.size} values do not fill rows of {nvar + 1}")
    rows = rows.reshape(-1, nvar + 1)
    return {"header": header, "start_time": start_time, "icol": icol, "t": rows[:, 0].copy(),
            "data": rows[:, 1:].copy()}
