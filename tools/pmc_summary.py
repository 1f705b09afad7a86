"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into profiles/pmc_summary.json.

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: FETCH_SIZE (KiB) reads exactly half of
the bytes for the 4/8/16-B-per-lane coalesced reads these kernels issue on gfx950 (calibrated by
tools/calibrate_pmc.hip, profiles/r01/pmc/calibration_*.csv; MI355X_MICROARCH.md §HBM), WRITE_SIZE is exact.
usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <num_ele> [out.json]
The summary carries bench.kernel_src_hash() of the tree it is written from: bench.py reports `traffic` only
while the kernel sources still hash the same (run it on the tree the passes were collected from)."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import kernel_src_hash  # noqa: E402  (keys the summary to the kernel build it was measured on)


def per_kernel(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        n = r["Kernel_Name"]
        key = ("shud_ele_kernel" if "ele_kernel" in n else "shud_riv_kernel" if "riv_kernel" in n else
               "shud_pack_kernel" if "pack_kernel" in n else None)
        if key:
            agg.setdefault(key, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    fd, wd, ne = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_summary.json"
    fe, wr = per_kernel(fd, "FETCH_SIZE"), per_kernel(wd, "WRITE_SIZE")
    res = {"num_ele": ne, "kernel_src_hash": kernel_src_hash(), "method": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 calibration)", "kernels": {}}
    for k in fe:
        rd, wb = 2 * fe[k] * 1024, wr.get(k, 0.0) * 1024
        res["kernels"][k] = {"read_bytes_per_launch": rd, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": rd + wb, "raw_fetch_kib": fe[k], "raw_write_kib": wr.get(k)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
