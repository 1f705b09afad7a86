"""Per-kernel averages of every counter in a rocprofv3 --pmc output directory (any counter set).
usage: python tools/pmc_counters.py <dir> [name-substring ...]  -> one line per (kernel, counter): dispatches, mean"""
import collections
import csv
import glob
import sys


def main():
    d, keys = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if keys and not any(k in n for k in keys):
                continue
            agg[(n.split("(")[0][:70], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (n, c), v in sorted(agg.items()):
        print(f"{n:70s} {c:24s} n={len(v):4d} mean={sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main()
