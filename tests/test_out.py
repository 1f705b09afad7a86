"""CPU: the Print_Ctrl restatement (tests/print_ctrl_py.py, the checker of include/shud_out.h) against the
reference's byte layout spelled out by hand (Model_Control.cpp:683-758, 893-960), and shudio.read_dat."""
import struct

import numpy as np

from print_ctrl_py import PrintCtrlPy
from shud_rhs.shudio import read_dat


def test_binary_layout_and_means(tmp_path):
    base = tmp_path / "ccw.eleysurf"
    p = PrintCtrlPy(base, 4, 60, iflux=0, start_time=1440, flag_io=[1, 0, 1, 1])
    vals = [np.array([1.0, 9.0, 2.0, 3.0]), np.array([3.0, 9.0, 4.0, 5.0]), np.array([0.5, 9.0, 0.25, 0.125])]
    for t, v in zip([30.0, 59.9995, 120.0], vals):      # 59.9995 + 0.001 floors to 60: interval ends
        p.print_data(v, t)
    p.close()
    raw = open(str(base) + ".dat", "rb").read()
    head = raw[:1024]
    assert head.startswith(b"# SHUD output\n# Radiation input mode: SWDOWN\n# Terrain radiation (TSR): OFF\n")
    assert head.rstrip(b"\0").endswith(b"lon=0.000000, lat=0.000000\n") and len(head) == 1024
    body = np.frombuffer(raw[1024:], dtype="<f8")
    want = [1440.0, 3.0, 1.0, 3.0, 4.0,                  # StartTime, NumVar, icol (1-based, masked column 2)
            0.0, (1.0 + 3.0) * (1.0 / 2), (2.0 + 4.0) * (1.0 / 2), (3.0 + 5.0) * (1.0 / 2),   # t = 60 - 60
            60.0, 0.5, 0.25, 0.125]                      # t = 120 - 60, one update
    assert body.tolist() == want
    d = read_dat(str(base) + ".dat")
    assert d["start_time"] == 1440.0 and d["icol"].tolist() == [1, 3, 4]
    assert d["t"].tolist() == [0.0, 60.0] and d["data"].shape == (2, 3)


def test_flux_tau_and_ascii(tmp_path):
    base = tmp_path / "ccw.rivqdown"
    p = PrintCtrlPy(base, 2, 1440, iflux=1, ascii=True, binary=True, radiation_input_mode=1, terrain_radiation=1,
                    solar_lonlat_mode="FIXED", lon=-120.5, lat=38.25)
    steps = np.arange(1, 145) * 10.0                     # 10-minute solver steps over one day
    rng = np.random.default_rng(1)
    v = rng.random((steps.size, 2))
    for t, x in zip(steps, v):
        p.print_data(x, t)
    p.close()
    acc = np.zeros(2)
    for x in v:
        acc += x
    mean = acc * (1440.0 / steps.size)
    d = read_dat(str(base) + ".dat")
    assert "SWNET" in d["header"] and "(TSR): ON" in d["header"] and "lon=-120.500000, lat=38.250000" in d["header"]
    assert d["t"].tolist() == [0.0] and np.array_equal(d["data"][0], mean)
    lines = open(str(base) + ".csv").read().splitlines()
    assert lines[0] == "# Timestamp semantics: left endpoint (t-Interval)" and lines[1] == "0\t 2\t 0"
    assert lines[6] == "Time_min \tX1 \tX2"
    assert lines[7] == "0.0\t" + "".join("%e\t" % x for x in mean)
    assert struct.unpack("<d", open(str(base) + ".dat", "rb").read()[1024:1032])[0] == 0.0
