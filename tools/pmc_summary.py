"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into profiles/pmc_summary.json.

FETCH_SIZE (KiB) tallies 64 B per L2 miss request on gfx950 (tools/calibrate_pmc.hip, profiles/r03/pmc_calib/):
a coalesced stream's 128-B lines count half their bytes (the blanket x2 of MI355X_MICROARCH.md §HBM), a
scattered access of <= 64 B counts one 64-B request (x1: random 64-B records read 1.00x, random 16-B pairs
4.00x).  Each kernel's single-use coalesced read streams C are known from its layout (COALESCED below), so
  HBM read bytes = C + (1024 * FETCH_SIZE - C / 2)      (the rest of the tally: scattered requests at x1)
and WRITE_SIZE * 1024 is exact for these stores.  `hbm_bytes_blanket_x2` keeps the old 2 * FETCH_SIZE form.
usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <num_ele> [out.json] [num_riv num_seg]
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


# single-use coalesced read streams, bytes per element / reach / segment (the packed layout, shud_dev.h):
# element kernel: meta 16, zz 16, y 24, {net_prep, pot_evap} 16, {pot_tran, ETP} 16, carried {u_satn, e_ic} 16,
# seg_first 4, the three edges' {edge, Dist2Nabor} 48, area 8 per element; per segment {length, Cwr} 16 + its
# reach index 4 (round 4: the reach's statics are a gathered per-reach record, counted with the scattered part;
# rounds 1-3 streamed a 48-B segment record)
# river kernel: its 64-B record, the 16-B index word rv_u, stage 8 per reach (round 4; rounds 1-3 also rv_i 16);
# segment positions 4 per segment.
COALESCED = {"shud_ele_kernel": (164, 0, 20), "shud_riv_kernel": (0, 88, 4)}


def main():
    fd, wd, ne = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_summary.json"
    nr, ns = (int(sys.argv[5]), int(sys.argv[6])) if len(sys.argv) > 6 else (972842, 5003338)   # syn-10M
    fe, wr = per_kernel(fd, "FETCH_SIZE"), per_kernel(wd, "WRITE_SIZE")
    res = {"num_ele": ne, "num_riv": nr, "num_seg": ns, "kernel_src_hash": kernel_src_hash(),
           "method": "read = C + (1024*FETCH_SIZE - C/2) with C the kernel's coalesced single-use read bytes "
                     "(FETCH_SIZE tallies 64 B per miss request: 1/2 of a coalesced 128-B line, 1x a scattered "
                     "<= 64-B access; profiles/r03/pmc_calib/), + 1024*WRITE_SIZE", "kernels": {}}
    for k in fe:
        pe, pr, ps = COALESCED.get(k, (0, 0, 0))
        c = pe * ne + pr * nr + ps * ns
        raw = fe[k] * 1024
        rd = c + (raw - c / 2) if raw >= c / 2 else 2 * raw
        wb = wr.get(k, 0.0) * 1024
        res["kernels"][k] = {"read_bytes_per_launch": rd, "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": rd + wb, "coalesced_read_bytes": c,
                             "hbm_bytes_blanket_x2": 2 * raw + wb, "raw_fetch_kib": fe[k], "raw_write_kib": wr.get(k)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
