"""Summarise tools/ele_phase_attr.sh: per library the element kernel's SQ counters (mean over dispatches, per
element wave = SQ total / ceil(NE/64); the QrivDown pre-pass waves ride in the same launch and are included) and
its median time from the interleaved A/B (abl.log), with the deltas against production.
usage: python tools/ele_phase_summary.py OUTDIR prod LIB1 LIB2 ..."""
import collections
import csv
import glob
import json
import sys

d, names = sys.argv[1], sys.argv[2:]
NE = 10001406
EW = -(-NE // 64)
DESC = {"prod": "production", "e1": "segment loop", "e2": "neighbour eff_kh (KsatH instead)", "e4": "edge loop",
        "e8": "f_etFlux", "e16": "satKfun (2 pow)", "e32": "report_w ballots", "e64": "infiltration + recharge",
        "a1": "pow -> mul", "a2": "cos -> id", "a4": "cbrt -> id", "a8": "IEEE div -> mul", "a16": "sqrt -> id"}
cnt = {}
for n in names:
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{d}/sq_{n}/**/*counter_collection.csv", recursive=True) + glob.glob(f"{d}/sq_{n}_counters.csv"):
        for r in csv.DictReader(open(f)):
            if "ele_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    cnt[n] = {k: sum(v) / len(v) for k, v in agg.items()}
tm = {}
try:
    last = [ln for ln in open(f"{d}/abl.log") if ln.startswith("{")][-1]
    med = json.loads(last)["ele_ms_median"]
    for k, v in med.items():
        tm["prod" if k == "pk" else k[4:] if k.startswith("lib:") else k] = v
except (OSError, IndexError, ValueError):
    pass
p = cnt.get("prod", {})
pt = tm.get("prod")
print(f"{'lib':6s} {'removed':34s} {'ele ms':>8s} {'d ms':>8s} {'VALU/ew':>9s} {'dVALU':>7s} {'TRANS/ew':>9s} "
      f"{'SALU/ew':>8s} {'VMEM/ew':>8s} {'LDS/ew':>7s}")
for n in names:
    c = cnt.get(n, {})
    v = c.get("SQ_INSTS_VALU", float("nan")) / EW
    pv = p.get("SQ_INSTS_VALU", float("nan")) / EW
    t = tm.get(n)
    print(f"{n:6s} {DESC.get(n, n):34s} {t if t else float('nan'):8.4f} "
          f"{(t - pt) if (t and pt) else float('nan'):+8.4f} {v:9.1f} {v - pv:+7.1f} "
          f"{c.get('SQ_INSTS_VALU_TRANS_F64', float('nan')) / EW:9.1f} {c.get('SQ_INSTS_SALU', float('nan')) / EW:8.1f} "
          f"{c.get('SQ_INSTS_VMEM', float('nan')) / EW:8.1f} {c.get('SQ_INSTS_LDS', float('nan')) / EW:7.1f}")
