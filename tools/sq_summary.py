"""Summarise tools/sq_counters.sh output per kernel (mean over dispatches): python tools/sq_summary.py gpurun_out"""
import csv, glob, sys, collections
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = "ele" if "ele_kernel" in n else "riv" if "riv_kernel" in n else None
        if k:
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    w = m.get("SQ_WAVES", 1)
    print(f"== {k}")
    for n in sorted(m):
        print(f"  {n:28s} {m[n]:16.0f}  per-wave {m[n] / w:10.1f}")
    if "GRBM_GUI_ACTIVE" in m and "SQ_INSTS_VALU" in m:
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        print(f"  kernel cycles (GRBM/8) {cyc:.0f};  VALU issue floor (4 cyc/wave-instr, 1024 SIMDs): "
              f"{m['SQ_INSTS_VALU'] * 4 / 1024:.0f} cyc = {m['SQ_INSTS_VALU'] * 4 / 1024 / cyc:.2f} of kernel")
