"""Regenerate the committed fixtures from the reference's own input data (run in the dev container,
where /root/reference exists; the GPU box only reads the outputs).

Writes:
  shud-up_amd/shud_rhs/data/ccw_tables.npz  ccw soil/geol/lc/river-type tables, calibration and the
                                            (iSoil, iGeol, iLC) rows of ccw.sp.att (synthetic meshes)
  tests/golden/ccw_model.npz, heihe_model.npz, qhh_model.npz  derived SoA after Model_Data::initialize()
                                            restated by shud_rhs.shudio (inputs of the parity tests) + .cfg.ic
                                            state (qhh: 688 lake elements, one lake, .lake.bathy table)
These are input DATA (the reference ships no outputs / golden vectors for the RHS: SURVEY §4).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "shud-up_amd"))
from shud_rhs import shudio  # noqa: E402

REF = "/root/reference/input"


def projects(names):
    for prj in names:
        m, ex = shudio.load_project(os.path.join(REF, prj), prj)
        m.step = {}
        m.save(os.path.join(HERE, f"{prj}_model.npz"))
        np.save(os.path.join(HERE, f"{prj}_y0.npy"), ex["y0"])
        print(prj, m.num_ele, m.num_riv, m.num_seg, m.num_lake, "sinks raised:", len(m.meta["raised"]))


def main():
    # ccw tables for the synthetic generator
    d = os.path.join(REF, "ccw")
    soil, _ = shudio.read_table(os.path.join(d, "ccw.para.soil"))
    geol, _ = shudio.read_table(os.path.join(d, "ccw.para.geol"))
    lc, _ = shudio.read_table(os.path.join(d, "ccw.para.lc"))
    with open(os.path.join(d, "ccw.sp.riv")) as f:
        rl = f.read().splitlines()
    _, nxt = shudio.read_table(rl, 0)
    rtype, _ = shudio.read_table(rl, nxt)
    att, _ = shudio.read_table(os.path.join(d, "ccw.sp.att"))
    cal = shudio.read_keyvals(os.path.join(d, "ccw.cfg.calib"))
    keys = sorted(cal)
    np.savez_compressed(os.path.join(ROOT, "shud-up_amd", "shud_rhs", "data", "ccw_tables.npz"),
                        soil=soil, geol=geol, lc=lc, rtype=rtype, att_rows=att[:, 1:4].astype(np.int64),
                        calib_keys=np.array(keys), calib_vals=np.array([cal[k] for k in keys]))
    projects(["ccw", "heihe", "qhh"])


if __name__ == "__main__":
    if len(sys.argv) > 1:
        projects(sys.argv[1:])
    else:
        main()
