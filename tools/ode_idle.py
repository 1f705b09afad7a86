"""GPU idle time inside the integrator section of a rocprofv3 kernel trace (bench.py's integrator measurement):
span from the first to the last integrator kernel, the union of kernel busy intervals, the gaps (host round trips,
launch latency) and the per-kernel totals.  usage: python tools/ode_idle.py KERNEL_TRACE_CSV"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "ode" in r["Kernel_Name"].lower()]
seg = rows[idx[0]:idx[-1] + 1]
t0, last, busy, gaps = int(seg[0]["Start_Timestamp"]), int(seg[0]["Start_Timestamp"]), 0, []
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > last:
        gaps.append(s - last)
    if e > last:
        busy += e - max(s, last)
    last = max(last, e)
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:60]
    agg[n][0] += 1
    agg[n][1] += (e - s) / 1e6
span = last - t0
print(f"span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms "
      f"({(span - busy) / span * 100:.2f} %), {len(seg)} kernels, {len(gaps)} gaps, median gap "
      f"{sorted(gaps)[len(gaps) // 2] / 1e3:.1f} us")
tot = sum(v[1] for v in agg.values())
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:60s} {v[0]:5d} {v[1]:8.3f} ms {v[1] / v[0] * 1e3:8.1f} us {v[1] / tot * 100:5.1f} %")
