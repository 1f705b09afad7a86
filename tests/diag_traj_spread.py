"""The ccw one-day trajectory's own divergence under rounding-level changes (tests/traj.py spread): CPU only.
usage: python tests/diag_traj_spread.py [out.json]  (the committed measurement: profiles/r04/traj/spread.json)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "oracle", "shud-up_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    from traj import spread
    res = {name: spread(mode) for mode, name in ((0, "serial"), (1, "omp"))}
    for name, r in res.items():
        print(name, json.dumps(r))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
