"""Achieved bandwidth of the integrator's vector kernels from a rocprofv3 kernel-stats CSV.
Algorithmic bytes per state entry of each kernel (shud_ode_kernels.hip: one read or write of each operand)
x NY entries / average duration.  Kernels whose byte count depends on the current order q (k_rescale,
k_complete) are priced at --q (the order the run mostly used).  usage:
  python tools/ode_bw.py kernel_stats.csv NY [--q 3]"""
import argparse
import csv
import re
import sys

# bytes per entry; callables take the order q
PER_ENTRY = {
    "k_ewt": lambda q: 16,
    "k_vsum_zero": lambda q: 24,
    "k_vsum": lambda q: 24,
    "k_scale_to": lambda q: 16,
    "k_residual": lambda q: 40,          # with ycor (the acor_zero call reads 32)
    "k_krylov_v0": lambda q: 24,
    "k_dq_work": lambda q: 32,
    "k_atimes": lambda q: 48,
    "k_mgs": lambda q: 32,               # w, Vprev, Vnext, w (the last pass of an iteration moves 24)
    "k_normalize": lambda q: 24,
    "k_newton_update": lambda q: 8 * (3 + 2),   # ewt, ycor, ~2 Krylov vectors, ycor
    "k_complete": lambda q: 8 * (1 + 2 * q),                # round 4: materializes zn[1..q] (eager: 1 + 2(q+1))
    "k_complete_ewt": lambda q: 24,         # round 4: acor, zn[0] -> ewt (zn[0] deferred too; --eager-zn0: 32;
                                            # eager complete: 8 * (1 + 2(q+1)) + 8)
    "k_rescale": lambda q: 16 * q,
    "k_eta_norms": lambda q: 32,
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("ny", type=int)
    ap.add_argument("--q", type=int, default=3)
    ap.add_argument("--eager-ycor", action="store_true", help="sources before the lazy ycor (predict stores ycor = 0)")
    ap.add_argument("--eager-complete", action="store_true",
                    help="sources before round 4's deferred cvCompleteStep (complete_ewt updates all of zn)")
    ap.add_argument("--eager-zn0", action="store_true", help="sources where complete_ewt still stores zn[0]")
    ap.add_argument("--copy-gbs", type=float, default=6400.0, help="the box's STREAM copy rate")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot_ns = tot_b = 0.0
    print(f"{'kernel':<22}{'calls':>7}{'avg us':>10}{'GB/s':>9}{'total ms':>10}")
    for r in rows:
        name = r["Name"]
        m = re.search(r"(k_\w+?)(?:<|\(|I)", name.replace("shud::ode::", ""))
        if "pascal" in name:
            mm = re.search(r"k_pascal<(\d), (true|false)(?:, (true|false))?", name)
            q = int(mm.group(1))
            fwd = mm.group(2) == "true"
            pend = mm.group(3) == "true"
            lazy = "--eager-ycor" not in sys.argv
            b = 8 * (2 * q + 1) + ((8 if lazy else 16) if fwd else 0)   # predict also writes y (+ ycor unless lazy)
            if pend:
                b += 16                         # the deferred completion: acor in, zn[q] out
            key = f"k_pascal<{q},{'pend' if pend else 'pred' if fwd else 'rest'}>"
        elif m and m.group(1) in PER_ENTRY:
            key = m.group(1)
            b = PER_ENTRY[key](a.q)
            if a.eager_complete and key == "k_complete":
                b = 8 * (1 + 2 * (a.q + 1))
            if a.eager_zn0 and key == "k_complete_ewt":
                b = 32
            if a.eager_complete and key == "k_complete_ewt":
                b = 8 * (1 + 2 * (a.q + 1)) + 8
        elif "k_finalize" in name:
            key, b = "k_finalize", 0
        else:
            continue
        avg = float(r["AverageNs"])
        calls = int(r["Calls"])
        tot_ns += float(r["TotalDurationNs"])
        tot_b += b * a.ny * calls
        gbs = b * a.ny / avg if b else float("nan")
        print(f"{key:<22}{calls:>7}{avg / 1e3:>10.1f}{gbs:>9.0f}{float(r['TotalDurationNs']) / 1e6:>10.2f}")
    print(f"integrator vector kernels total {tot_ns / 1e6:.2f} ms, {tot_b / 1e9:.1f} GB algorithmic "
          f"({tot_b / tot_ns:.0f} GB/s average; {tot_b / a.copy_gbs / 1e6:.2f} ms at {a.copy_gbs:.0f} GB/s)")


if __name__ == "__main__":
    main()
