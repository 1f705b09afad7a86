"""tools/pmc_summary.py: the per-pattern FETCH_SIZE model (profiles/r03/pmc_calib/) on synthetic counter files —
coalesced single-use streams tallied at half their bytes, the rest of the tally counted once."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(d, counter, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for name, v in rows:
            w.writerow({"Kernel_Name": name, "Counter_Name": counter, "Counter_Value": v})


def test_pmc_summary_model(tmp_path):
    ne, nr, ns = 1000, 100, 500
    c_ele = 164 * ne + 20 * ns
    c_riv = 88 * nr + 4 * ns
    ele = "void shud::shud_ele_kernel_packed<0, false>(x)"
    riv = "void shud::shud_riv_kernel_packed<0, false, 0>(x)"
    # element: coalesced tally C/2 plus 10 KiB of scattered requests; river: C/2 plus 40 KiB; two launches each
    fe = [(ele, (c_ele / 2 + 10240) / 1024), (ele, (c_ele / 2 + 10240) / 1024),
          (riv, (c_riv / 2 + 40960) / 1024), (riv, (c_riv / 2 + 40960) / 1024)]
    wr = [(ele, 48.0), (ele, 48.0), (riv, 1.0), (riv, 1.0)]
    _write(tmp_path / "f", "FETCH_SIZE", fe)
    _write(tmp_path / "w", "WRITE_SIZE", wr)
    out = tmp_path / "s.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path / "f"),
                    str(tmp_path / "w"), str(ne), str(out), str(nr), str(ns)], check=True, capture_output=True)
    s = json.load(open(out))
    k = s["kernels"]
    assert abs(k["shud_ele_kernel"]["read_bytes_per_launch"] - (c_ele + 10240)) < 1e-6
    assert abs(k["shud_ele_kernel"]["hbm_bytes_per_launch"] - (c_ele + 10240 + 48 * 1024)) < 1e-6
    assert abs(k["shud_ele_kernel"]["hbm_bytes_blanket_x2"] - (c_ele + 2 * 10240 + 48 * 1024)) < 1e-6
    assert abs(k["shud_riv_kernel"]["read_bytes_per_launch"] - (c_riv + 40960)) < 1e-6
    assert s["num_riv"] == nr and s["num_seg"] == ns and len(s["kernel_src_hash"]) == 16
