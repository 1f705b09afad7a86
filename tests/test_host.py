"""The C++ host above the device path (libshud_host.so, include/shud_host.h), on CPU.

* Readers + Model_Data::initialize + LoadIC restated in C++ equal the Python restatement (shud_rhs/shudio.py,
  which built the committed fixtures) bit for bit on the reference's own inputs (ccw, heihe with END 9000, qhh;
  skipped where /root/reference is absent) and on a synthetic project written in SHUD text formats.
* Forcing: zero-order hold of every series exactly as _TimeSeriesData::movePointer/getX (TimeSeriesData.cpp),
  the missing-data exit, and the TSR bucket (MD_ET.cpp:60-136) with solar samples equal to an independent
  pure-Python restatement of solarPosition/TimeContext (tests/solar_py.py) bit for bit.
* Control_Data keys and the print-control list of initialize_output (MD_initialize.cpp:246-345).
Parity is unpinned by the reference itself (no SUNDIALS build): the pins are the two
restatements agreeing and the reference's own input files.
"""
import math
import os

import numpy as np
import pytest

import solar_py
from shud_rhs import abi, host, shudio, synth

REF_INPUT = "/root/reference/input"


def _diff(a, b):
    bad = []
    for grp in ("ele", "par", "riv"):
        da, db = getattr(a, grp), getattr(b, grp)
        for k in db:
            if k in da and not np.array_equal(da[k], db[k]):
                bad.append(f"{grp}.{k}")
    for k in ("nabr", "ibc", "iss", "riv_down", "riv_bc", "seg_ele", "seg_riv", "seg_length", "seg_cwr"):
        if not np.array_equal(getattr(a, k), getattr(b, k)):
            bad.append(k)
    if a.num_lake != b.num_lake:
        bad.append("num_lake")
    elif a.num_lake:
        for k in ("lake_bathy_off", "lake_bathy_y", "lake_bathy_a"):
            if not np.array_equal(getattr(a, k), getattr(b, k)):
                bad.append(k)
    return bad


@pytest.mark.parametrize("prj,end", [("ccw", -1), ("heihe", 9000), ("qhh", -1)])
def test_reader_matches_python_restatement(prj, end):
    indir = os.path.join(REF_INPUT, prj)
    if not os.path.isdir(indir):
        pytest.skip("reference inputs absent")
    P = host.Project(indir, prj, cwd="/root/reference", end_day=end)
    m = P.model()
    ref, ex = shudio.load_project(indir, prj)
    assert _diff(m, ref) == []
    assert np.array_equal(P.array("y0"), ex["y0"])
    c = P.control()
    assert c["lakeon"] == (ref.num_lake > 0)
    # the committed fixture (made from the Python restatement) agrees too
    from conftest import load_fixture
    fm, fy = load_fixture(prj)
    assert _diff(m, fm) == [], "fixture"
    assert np.array_equal(P.array("y0"), fy)


def test_synthetic_project_round_trip(tmp_path):
    m = synth.write_project(str(tmp_path), "syn", 1500, days=1.0)
    P = host.Project(str(tmp_path), "syn", cwd=str(tmp_path))
    hm = P.model()
    assert _diff(hm, m) == []
    ref, ex = shudio.load_project(str(tmp_path), "syn")
    assert _diff(hm, ref) == []
    assert np.array_equal(P.array("y0"), ex["y0"])
    et = P.et_model()
    assert np.array_equal(et.arrays["z_surf"], m.ele["z_surf"])
    assert np.array_equal(et.arrays["veg_frac"], m.par["VegFrac"])
    # PressureElevation on the final (rmSinks) surface, Element.cpp:222
    fixp = [101.325 * math.pow((293. - 0.0065 * z) / 293, 5.26) for z in m.ele["z_surf"]]   # glibc pow
    assert np.array_equal(et.arrays["fix_pressure"], fixp)
    n = np.stack([et.arrays["nx"], et.arrays["ny"], et.arrays["nz"]])
    assert np.allclose((n * n).sum(0), 1.0, rtol=0, atol=1e-15) and np.all(n[2] >= 0)


def test_control_and_print_controls_ccw():
    indir = os.path.join(REF_INPUT, "ccw")
    if not os.path.isdir(indir):
        pytest.skip("reference inputs absent")
    P = host.Project(indir, "ccw", cwd="/root/reference")
    c = P.control()
    # ccw.cfg.para: MAX_SOLVER_STEP 10, LSM_STEP 60, INIT_SOLVER_STEP 1, END 1827, RELTOL/ABSTOL 1e-4
    assert (c["solver_step"], c["et_step"], c["init_step"], c["reltol"], c["abstol"]) == (10, 60, 1, 1e-4, 1e-4)
    assert c["end_time"] == 1827 * 1440 and c["num_steps"] == 1827 * 144
    assert (c["forc_start_time"], c["num_forc"], c["terrain_radiation"]) == (20000101, 1, 1)
    assert (c["solar_lon_deg"], c["solar_lat_deg"]) == (-122.71, 39.195)
    outs = P.outputs("/tmp/out")
    names = [os.path.basename(o["basename"]) for o in outs]
    # initialize_output order for ccw's DT_* keys (all 1440)
    assert names == ["ccw.eleysnow", "ccw.eleysurf", "ccw.eleyunsat", "ccw.eleygw", "ccw.elevprcp",
                     "ccw.elevnetprcp", "ccw.elevetp", "ccw.eleveta", "ccw.elevrech", "ccw.eleqsub",
                     "ccw.eleqsurf", "ccw.elevinfil", "ccw.elevexfil", "ccw.elevetic", "ccw.elevettr",
                     "ccw.elevetev", "ccw.rn_h", "ccw.rn_t", "ccw.rn_factor", "ccw.rivqup", "ccw.rivqdown",
                     "ccw.rivqsub", "ccw.rivqsurf", "ccw.rivystage"]
    assert all(o["interval"] == 1440 for o in outs)
    flux = {n for n, o in zip(names, outs) if o["iflux"]}
    assert "ccw.eleysurf" not in flux and "ccw.rn_factor" not in flux and "ccw.rivqdown" in flux


def _csv_rows(path):
    rows = []
    with open(path) as f:
        f.readline()
        f.readline()
        for line in f:
            t = line.split()
            if t:
                rows.append([float(v) for v in t])
    a = np.array(rows)
    a[:, 0] = a[:, 0] * 1440.0
    return a


def test_forcing_zero_order_hold(tmp_path):
    synth.write_project(str(tmp_path), "syn", 600, days=3.0, forcing_dt_min=180.0)
    P = host.Project(str(tmp_path), "syn", cwd=str(tmp_path))
    wx = _csv_rows(os.path.join(tmp_path, "forcing.csv"))
    lai = _csv_rows(os.path.join(tmp_path, "syn.tsd.lai"))
    for t in np.arange(0.0, 3 * 1440.0, 60.0):
        f = P.forcing(t, t + 60.0)
        k = np.nonzero(wx[:, 0] <= t)[0][-1]
        assert np.array_equal(f.station[0], wx[k]), t
        kl = np.nonzero(lai[:, 0] <= t)[0][-1]
        assert np.array_equal(f.lai_row, lai[kl]), t
        assert f.station_z[0] == -9999.0


def test_forcing_missing_data_exit(tmp_path):
    synth.write_project(str(tmp_path), "syn", 600, days=1.0)
    P = host.Project(str(tmp_path), "syn", cwd=str(tmp_path))
    last = _csv_rows(os.path.join(tmp_path, "forcing.csv"))[-1, 0]
    P.forcing(last + 1440.0, last + 1500.0)                 # within a day of the last row: held
    with pytest.raises(RuntimeError, match="missing forcing data"):
        P.forcing(last + 1441.5, last + 1500.0)             # TimeSeriesData.cpp:296-300


def test_solar_position_kat(tmp_path):
    synth.write_project(str(tmp_path), "syn", 600, days=1.0)
    P = host.Project(str(tmp_path), "syn", cwd=str(tmp_path))
    rng = np.random.default_rng(7)
    ts = np.concatenate([rng.uniform(-5e5, 5e6, 300), np.arange(0, 2 * 1440, 37.5), [59 * 1440 + 720.0]])
    lats = [-90.0, -45.3, 0.0, 39.195, 66.6, 90.0, 120.0]
    lons = [-200.0, -122.71, 0.0, 100.95, 179.9, 181.0, 540.5]
    n = 0
    for t in ts:
        for la in lats:
            for lo in lons[:3] if n % 2 else lons:
                got = P.solar(t, la, lo, 0.0)
                ref = solar_py.solar_position(20000101, float(t), la, lo, 0.0)
                assert got == ref, (t, la, lo, got, ref)
                n += 1
    assert solar_py.julian_day(20000101, 59 * 1440.0) == 60 and solar_py.julian_day(20000101, 366 * 1440.0) == 1


def test_tsr_buckets(tmp_path):
    # forcing every 180 min, ET step 60 min: a new interval every third step -> RECOMPUTE, CACHED, CACHED
    synth.write_project(str(tmp_path), "syn", 600, days=2.0, forcing_dt_min=180.0)
    P = host.Project(str(tmp_path), "syn", cwd=str(tmp_path))
    c = P.control()
    wx = _csv_rows(os.path.join(tmp_path, "forcing.csv"))
    modes, dens = [], []
    for t in np.arange(0.0, 2 * 1440.0, 60.0):
        f = P.forcing(t, t + 60.0)
        modes.append(f.tsr_mode)
        dens.append(f.tsr_den)
        k = np.nonzero(wx[:, 0] <= t)[0][-1]
        t0, t1 = wx[k, 0], wx[k + 1, 0]
        sx, sy, sz, wd, den = solar_py.tsr_samples(20000101, t0, t1, 60, c["solar_lat_deg"], c["solar_lon_deg"])
        assert f.tsr is not None
        assert np.array_equal(f.tsr[0], sx) and np.array_equal(f.tsr[1], sy)
        assert np.array_equal(f.tsr[2], sz) and np.array_equal(f.tsr[3], wd) and f.tsr_den == den, t
    assert modes[:6] == [abi.SHUD_TSR_RECOMPUTE, abi.SHUD_TSR_CACHED, abi.SHUD_TSR_CACHED] * 2
    assert max(dens) > 0 and min(dens) == 0.0                # daytime and night-time intervals both covered


def test_boundary_condition_rows_and_cfg_output(tmp_path):
    """read_bcEle1/2, read_bcRiv1/2 (MD_readin.cpp:959-982) with the zero-order hold f_update reads through
    getX (MD_update.cpp:114-125, 145-160); read_cfgout's column flags (MD_readin.cpp:25-104)."""
    synth.write_project(str(tmp_path), "syn", 900, days=1.0, bc=True, cfg_output=True)
    P = host.Project(str(tmp_path), "syn", cwd=str(tmp_path))
    m = P.model()
    tabs = {k: _csv_rows(os.path.join(tmp_path, f"syn.tsd.{e}"))
            for k, e in (("ele_ybc", "ebc1"), ("ele_qbc", "ebc2"), ("riv_ybc", "rbc1"), ("riv_qbc", "rbc2"))}
    for t in np.arange(0.0, 1440.0, 45.0):
        P.forcing(t, t + 45.0)
        rows = P.bc_rows()
        assert set(rows) == set(tabs)
        for k, tab in tabs.items():
            r = np.nonzero(tab[:, 0] <= t)[0][-1]
            assert np.array_equal(rows[k], tab[r]), (k, t)
    assert sorted(set(m.ibc.tolist())) == [-2, -1, 0, 1, 2] and sorted(set(m.riv_bc.tolist())) == [-1, 0, 1]
    outs = P.outputs(str(tmp_path / "out"))
    ele = next(o for o in outs if o["basename"].endswith(".eleygw"))
    riv = next(o for o in outs if o["basename"].endswith(".rivystage"))
    NE, NR = m.num_ele, m.num_riv
    off = np.arange(0, NE, max(1, NE // 7))
    want = np.ones(NE, dtype=np.int32)
    want[off] = 0
    assert np.array_equal(ele["flag_io"], want)
    want = np.zeros(NR, dtype=np.int32)
    want[np.arange(0, NR, max(1, NR // 5))] = 1
    assert np.array_equal(riv["flag_io"], want)
