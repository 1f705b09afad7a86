"""The C++ host driver (shud-up_amd/shud_gpu: SHUD()'s loop, src/Model/shud.cpp:86-140) end to end on the GPU.

A synthetic project in the reference's text formats (shud_rhs.synth.write_project: mesh, attributes, parameter
tables, rivers, calibration, cfg.para / cfg.ic, forcing list + csv, LAI, MF) is run by
  * shud_gpu (C++: libshud_host readers/init/forcing + the device RHS, ET prelude, integrator and outputs), and
  * the Python driver (ShudSolver + runtime.Output) over the same libshud_host project;
every .dat output must be byte-identical.  A hand-driven device run of the same loop is checked against the
CPU oracle chain (oracle ET prelude + oracle RHS + oracle integrator, fed the C++ host's forcing rows) over the
first hour, as tests/test_gpu_ode.py does for synthetic forcing: within 1e-6 of the solver's error weight
(parity unpinned by the reference itself)."""
import glob
import os
import subprocess

import numpy as np
import pytest

import oracle
from conftest import PKG_DIR, assert_close
from shud_rhs import abi, host, shudio, synth
from shud_rhs import runtime as rt
from shud_rhs.solver import SolverControl, ShudSolver

pytestmark = pytest.mark.gpu
SHUD_GPU = os.path.join(PKG_DIR, "shud_gpu")
LONLAT = {0: "FORCING_FIRST", 1: "FORCING_MEAN", 2: "FIXED"}


def _ctl(c):
    return SolverControl(reltol=c["reltol"], abstol=c["abstol"], init_step=c["init_step"], max_step=c["max_step"],
                         et_step=c["et_step"], start=c["start_time"])


def _device_model(P):
    m = P.model()
    h = rt.RhsHandle(m, mode=abi.SHUD_MODE_SERIAL)
    h.et_attach(P.et_model())
    h.et_set_state(P.array("y_is"), P.array("y_snow"))
    h.set_step_inputs(step={"u_satn": np.zeros(m.num_ele)})      # shud_gpu.cpp: first updateforcing's u_satn
    return m, h


@pytest.mark.parametrize("case", ["plain", "bc_substep"])
def test_shud_gpu_matches_python_driver(tmp_path, case):
    """plain: 10-min solver steps, ET every step.  bc_substep: element/river boundary-condition tables
    (.tsd.ebc1/.ebc2/.rbc1/.rbc2 rows through shud_project_bc_rows), a .cfg.output column selection, and ET
    sub-stepping (ETStep 10 < SolverStep 30: CVodeSetStopTime per ET step, shud.cpp:86-87,112-115)."""
    src = tmp_path / "in"
    if case == "plain":
        synth.write_project(str(src), "syn", 2000, days=1.0, max_step=10.0, et_step=60.0, dt_out=60)
    else:
        synth.write_project(str(src), "syn", 2000, days=1.0, max_step=30.0, et_step=10.0, dt_out=60, bc=True,
                            cfg_output=True)
    out_c, out_p = tmp_path / "out_cpp", tmp_path / "out_py"
    r = subprocess.run([SHUD_GPU, "-o", str(out_c), "-C", str(src), str(src), "syn"], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "RHS" in r.stdout

    P = host.Project(str(src), "syn", cwd=str(src))
    c = P.control()
    m, h = _device_model(P)
    sv = ShudSolver(h, P.array("y0"), _ctl(c))
    h.prepare_outputs()
    out = rt.Output(stream=h.stream())
    os.makedirs(out_p)
    decl = P.outputs(str(out_p))
    for d in decl:
        p, n = h.device_array(d["array"])
        if d["column"] >= 0:
            p += 8 * d["column"] * m.num_ele
        out.add(d["basename"], p, d["n_all"], d["interval"], d["iflux"], start_time=c["forc_start_time"],
                flag_io=d["flag_io"],
                binary=bool(c["binary"]), ascii=bool(c["ascii"]), radiation_input_mode=c["radiation_input_mode"],
                terrain_radiation=c["terrain_radiation"], solar_lonlat_mode=LONLAT[c["solar_lonlat_mode"]],
                lon=c["solar_lon_deg"], lat=c["solar_lat_deg"])
    def forcing(t, tout):                       # shud_gpu.cpp: forcing rows, then the BC rows, then ET
        f = P.forcing(t, tout)
        bc = P.bc_rows()
        if bc:
            h.set_step_inputs(step={}, bc_tables=bc)
        return f

    assert (len(P.bc_rows()) == 4) == (case == "bc_substep")
    t, _ = sv.run(c["num_steps"], forcing=forcing, output=out)
    assert abs(t - c["end_time"]) < 1e-6
    out.close()
    files = sorted(os.path.basename(f) for f in glob.glob(str(out_c / "*.dat")))
    assert len(files) == len(decl) == 24
    assert files == sorted(os.path.basename(f) for f in glob.glob(str(out_p / "*.dat")))
    for f in files:
        a, b = open(out_c / f, "rb").read(), open(out_p / f, "rb").read()
        assert a == b, f
        d = shudio.read_dat(str(out_c / f))
        assert d["t"].size == 24 and np.all(np.isfinite(d["data"])), f
        if case != "plain" and ".riv" in f:
            assert d["data"].shape[1] < m.num_riv                  # cfg.output selection
        assert np.array_equal(d["t"], np.arange(24) * 60.0)
    if case == "plain":
        gw = shudio.read_dat(str(out_c / "syn.eleygw.dat"))["data"]
        assert np.abs(gw - P.array("y0")[2 * m.num_ele:3 * m.num_ele]).max() < 1.0    # one day moves gw < 1 m
    sv.close()
    h.close()


def test_device_loop_vs_oracle_chain_first_hour(tmp_path):
    synth.write_project(str(tmp_path), "syn", 2000, days=1.0, max_step=10.0, et_step=60.0, dt_out=60)
    P = host.Project(str(tmp_path), "syn", cwd=str(tmp_path))
    c = P.control()
    ctl = _ctl(c)
    y0 = P.array("y0")
    m, h = _device_model(P)
    etm = P.et_model()
    oe = oracle.OracleEt(etm)
    oe.set_state(P.array("y_is"), P.array("y_snow"))
    r = oracle.OracleRhs(m, abi.SHUD_MODE_SERIAL)
    r.set_step_inputs(step={"u_satn": np.zeros(m.num_ele)})
    d = rt.OdeSolver(h, ctl.start, y0, ctl.reltol, ctl.abstol, ctl.init_step, ctl.max_step, ctl.min_step,
                     ctl.max_num_steps)
    o = oracle.OracleOde(r, ctl.start, y0, ctl.reltol, ctl.abstol, ctl.init_step, ctl.max_step, ctl.min_step,
                         ctl.max_num_steps)
    t = tnext = ctl.start
    for i in range(6):                                   # 10-minute solver steps, one ET step (60 min)
        tnext += ctl.solver_step
        while t + 1e-10 < tnext:
            tout = tnext
            f = P.forcing(t, tout)
            assert h.et_step(f) == abi.SHUD_OK
            assert oe.step(f) == (0, -1)
            got = h.et_get()
            for key in ["qEleNetPrep", "qPotEvap", "qPotTran", "qEleETP", "qEleE_IC", "rn_factor"]:
                assert_close(got[key], oe.get()[key], what=f"ET {key} t={t}")
            r.set_step_inputs(step=dict(net_prep=got["qEleNetPrep"], pot_evap=got["qPotEvap"],
                                        pot_tran=got["qPotTran"], etp=got["qEleETP"], lai=got["t_lai"],
                                        fu_surf=got["fu_surf"], fu_sub=got["fu_sub"], e_ic=got["qEleE_IC"]))
            fd, td, yd = d.solve(tout)
            fo, t, yo = o.solve(tout)
            assert fd == fo == 0 and td == t
            err = np.abs(yd - yo)
            tol = 1e-6 * (ctl.reltol * np.abs(yo) + ctl.abstol)
            assert np.all(err <= tol), f"t={t}: max err {err.max():.3e}"
    sd, so = d.stats(), o.stats()
    for key in ["nst", "nfe", "nni", "nli", "netf", "ncfn"]:
        assert sd[key] == so[key], (key, sd[key], so[key])
    d.close()
    h.close()


@pytest.mark.parametrize("parts,lake", [(2, False), (4, False), (8, False), (2, True), (3, True)])
def test_shud_gpu_rhs_partition_check(tmp_path, parts, lake):
    """shud_gpu --rhs-check K: the C++ host partitions a synthetic project (C++ partitioner + planner), drives K
    partitioned RHS handles on one GPU with the halo moved by D2D copies and the ET prelude run on every local
    mesh, and compares every owned DY with the unpartitioned handle's: zero mismatched entries (bit-identical).
    lake: a project with one lake (200 lake elements); the owned state of the lake's rank carries the lake stage
    after its reaches ([sf|us|gw|riv|lake]) and the lake's DY is compared too."""
    import json
    src = tmp_path / "in"
    synth.write_project(str(src), "syn", 30000, days=1.0, max_step=10.0, et_step=60.0, dt_out=60, lake=lake)
    r = subprocess.run([SHUD_GPU, "--rhs-check", str(parts), "--evals", "6", "-C", str(src), str(src), "syn"],
                       capture_output=True, text=True, timeout=240)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('{"shud_gpu_rhs_check"')]
    assert r.returncode == 0 and line, r.stdout + r.stderr
    res = json.loads(line[-1])["shud_gpu_rhs_check"]
    assert res["parts"] == parts and res["evals"] == 6 and res["mismatched_entries"] == 0, res
    assert res["max_ghost_ele"] > 0 and res["imbalance"] < 1.05


@pytest.mark.parametrize("lake", [False, True])
def test_shud_gpu_rhs_bench_single_rank(tmp_path, lake):
    """shud_gpu --rhs-bench with WORLD_SIZE = 1 (the N > 1 mode runs one process per GPU over RCCL); with a lake
    the device state holds the lake stage after the reaches."""
    import json
    src = tmp_path / "in"
    synth.write_project(str(src), "syn", 30000, days=1.0, max_step=10.0, et_step=60.0, dt_out=60, lake=lake)
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([SHUD_GPU, "--rhs-bench", "--evals", "20", "-o", str(tmp_path / "o"), "-C", str(src),
                        str(src), "syn"], capture_output=True, text=True, timeout=240, env=env)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('{"shud_gpu_rhs_bench"')]
    assert r.returncode == 0 and line, r.stdout + r.stderr
    res = json.loads(line[-1])["shud_gpu_rhs_bench"]
    assert res["evals"] == 20 and res["exit_code"] == 0 and res["ms_per_eval"] > 0
