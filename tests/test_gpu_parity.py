"""GPU parity: libshud_rhs.so (HIP, gfx950) against the CPU restatement oracle on identical inputs.

Tolerance |gpu - ref| <= 1e-12 |ref| + 1e-15 per state (conftest.RTOL/ATOL).  Every case
runs several successive calls per state because the serial RHS is stateful (qEleE_IC, u_satn).
"""
import numpy as np
import pytest

import cases
from conftest import assert_close
from shud_rhs import abi, workload

pytestmark = pytest.mark.gpu


def _runtime():
    from shud_rhs import runtime
    return runtime


@pytest.fixture(params=["packed", "soa"])
def layout(request, monkeypatch):
    """Both device layouts: the packed class-table kernel (default when the mesh qualifies) and the plain
    SoA kernel (SHUD_RHS_PACKED=0)."""
    monkeypatch.setenv("SHUD_RHS_PACKED", "1" if request.param == "packed" else "0")
    return request.param


def _compare_sequence(m, ys, mode, oracle_mod, ncalls=3, diag=True, label="", layout=None):
    rt = _runtime()
    g = rt.RhsHandle(m, mode=mode)
    if layout is not None:
        assert g.layout()["packed"] == (layout == "packed"), g.layout()
    o = oracle_mod.OracleRhs(m, mode)
    g.set_step_inputs()
    o.set_step_inputs()
    worst = 0.0
    for si, y in enumerate(ys):
        for c in range(ncalls):
            ref, code, _, _ = o.eval(0.0, y)
            assert code == 0, f"{label}: oracle exit {code}"
            got = g.eval(0.0, y)
            _, rel = assert_close(got, ref, what=f"{label} state {si} call {c}")
            worst = max(worst, rel)
    if diag:
        dg, do = g.diagnostics(), o.diagnostics()
        for k in abi.FLUXOUT_ORDER:
            if mode == abi.SHUD_MODE_OMP and k in ("q_es", "q_eu", "q_eg", "q_tu", "q_tg", "q_eta", "i_beta"):
                continue
            # the *_tot / qe2r / qriv sums are near-cancelling sums of much larger fluxes: like DY they may
            # carry the OCML-vs-glibc ulps of their terms (conftest.assert_close `blocks`, <= 0.1 % of entries)
            sums = k in ("qele_surf_tot", "qele_sub_tot", "qe2r_surf", "qe2r_sub", "qriv_up", "qriv_surf", "qriv_sub")
            assert_close(dg[k], do[k], what=f"{label} diag {k}", blocks=[slice(None)] if sums else None)
    assert g.num_calls() == len(ys) * ncalls
    g.close()
    return worst


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_ccw(mode, oracle_mod, layout):
    m, y0 = cases.ccw()
    _compare_sequence(m, cases.states(m, y0), mode, oracle_mod, label="ccw", layout=layout)


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_heihe(mode, oracle_mod, layout):
    m, y0 = cases.heihe()
    _compare_sequence(m, cases.states(m, y0), mode, oracle_mod, label="heihe", layout=layout)


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_river_junctions(mode, oracle_mod, layout):
    """Junction shapes of the river kernel's index word (shud_dev.h rv_u): reaches with 0, 1, 2 upstream reaches
    inline, and 3, 5 and 14 through the up_idx slots (two 8-slot batches).  Headwater reaches of a small synthetic
    network are rewired into two targets (a headwater is never on a target's downstream path: no cycles);
    the junction sums keep ascending upstream order (MD_f.cpp:236-240) like the oracle."""
    from shud_rhs import synth
    m = synth.synth_model(20000)
    down = m.riv_down.astype(np.int64)
    nup = np.bincount(down[down >= 0], minlength=m.num_riv)
    heads = np.nonzero(nup == 0)[0]
    t_big = int(np.nonzero((nup == 0) & (down >= 0))[0][0])        # a headwater with a downstream reach
    t_three = int(np.nonzero(nup == 1)[0][0])
    movers = [h for h in heads if h not in (t_big, t_three)]
    down[movers[:14]] = t_big
    down[movers[14:16]] = t_three
    m.riv_down = down.astype(np.int32)
    nup = np.bincount(down[down >= 0], minlength=m.num_riv)
    assert nup[t_big] == 14 and nup[t_three] == 3 and {0, 1, 2, 5} <= set(nup.tolist())
    _compare_sequence(m, cases.states(m, None, 2, seed=21), mode, oracle_mod, label="junctions", layout=layout)


def _junction_model():
    from shud_rhs import synth
    m = synth.synth_model(20000)
    down = m.riv_down.astype(np.int64)
    nup = np.bincount(down[down >= 0], minlength=m.num_riv)
    heads = np.nonzero(nup == 0)[0]
    t_big = int(np.nonzero((nup == 0) & (down >= 0))[0][0])
    t_three = int(np.nonzero(nup == 1)[0][0])
    movers = [h for h in heads if h not in (t_big, t_three)]
    down[movers[:14]] = t_big
    down[movers[14:16]] = t_three
    m.riv_down = down.astype(np.int32)
    return m, None


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_river_paths_bit_identical(mode, oracle_mod, monkeypatch):
    """The river kernel's build paths give the same bits: QrivDown from the element launch's pre-pass slots
    (default) or recomputed from the reach records (SHUD_RHS_QD=0), with 6 or 8 segments per gather batch
    (SHUD_RIV_SB; the handle otherwise picks one from the mesh).  ccw, heihe, the branch variant and the junction
    shapes, 3 stateful calls on 2 states, every river diagnostic; one path also against the oracle."""
    rt = _runtime()
    for label, (m, y0) in (("ccw", cases.ccw()), ("heihe", cases.heihe()), ("variant", cases.variant()),
                           ("junctions", _junction_model())):
        ys = cases.states(m, y0, 2, seed=5)
        outs = {}
        for qd in ("1", "0"):
            for sb in ("6", "8"):
                monkeypatch.setenv("SHUD_RHS_QD", qd)
                monkeypatch.setenv("SHUD_RIV_SB", sb)
                g = rt.RhsHandle(m, mode=mode)
                assert g.layout()["packed"]
                g.set_step_inputs()
                seq = [g.eval(0.0, y) for y in ys for _ in range(3)]
                dg = g.diagnostics()
                outs[(qd, sb)] = (seq, {k: dg[k] for k in ("qriv_down", "qriv_up", "qriv_surf", "qriv_sub")})
                g.close()
        ref_seq, ref_dg = outs[("0", "8")]
        for key, (seq, dg) in outs.items():
            for c, (a, b) in enumerate(zip(seq, ref_seq)):
                assert np.array_equal(a, b, equal_nan=True), f"{label} QD={key[0]} SB={key[1]} call {c}"
            for k in dg:
                assert np.array_equal(dg[k], ref_dg[k], equal_nan=True), f"{label} QD={key[0]} SB={key[1]} {k}"
        o = oracle_mod.OracleRhs(m, mode)
        o.set_step_inputs()
        seq = outs[("1", "6")][0]
        k = 0
        for si, y in enumerate(ys):
            for c in range(3):
                assert_close(seq[k], o.eval(0.0, y)[0], what=f"{label} QD SB6 state {si} call {c}")
                k += 1
    monkeypatch.delenv("SHUD_RHS_QD")
    monkeypatch.delenv("SHUD_RIV_SB")


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_variant_branches(mode, oracle_mod, layout):
    m, y = cases.variant()
    _compare_sequence(m, [y] + cases.states(m, None, 2, seed=9), mode, oracle_mod, label="variant", layout=layout)


def test_step_inputs_update(oracle_mod, layout):
    """A new ET step (set_step_inputs) mid-sequence, carried state overridden then carried on."""
    rt = _runtime()
    m, y0 = cases.ccw()
    g, o = rt.RhsHandle(m), oracle_mod.OracleRhs(m, 0)
    g.set_step_inputs(); o.set_step_inputs()
    y = workload.random_state(m, seed=3)
    for step_seed in [21, 22]:
        st = workload.random_step_inputs(m, seed=step_seed)
        g.set_step_inputs(st); o.set_step_inputs(st)
        for c in range(2):
            assert_close(g.eval(1.0, y), o.eval(1.0, y)[0], what=f"step {step_seed} call {c}")
    # partial update (NULL arrays keep the previous values)
    st = {"net_prep": np.full(m.num_ele, 1e-5)}
    g.set_step_inputs(st); o.set_step_inputs(st)
    assert_close(g.eval(2.0, y), o.eval(2.0, y)[0], what="partial step update")


def test_device_pointer_eval(oracle_mod, layout):
    rt = _runtime()
    m, y0 = cases.ccw()
    g, o = rt.RhsHandle(m), oracle_mod.OracleRhs(m, 0)
    g.set_step_inputs(); o.set_step_inputs()
    ny = m.num_y
    dy_ptr, dd_ptr = g.device_alloc(8 * ny), g.device_alloc(8 * ny)
    try:
        for c in range(3):
            g.h2d(dy_ptr, y0)
            g.eval_device(0.0, dy_ptr, dd_ptr)
            got = g.d2h(np.zeros(ny), dd_ptr)
            assert_close(got, o.eval(0.0, y0)[0], what=f"device eval call {c}")
        ms, per = g.time_kernels(0.0, dy_ptr, dd_ptr, 3)
        assert ms > 0 and per["shud_ele_kernel"] > 0
    finally:
        g.device_free(dy_ptr)
        g.device_free(dd_ptr)


def test_cvrhs_entry(oracle_mod):
    """shud_rhs_cvrhs: the CVRhsFn body (user_data = handle) used by the INTEGRATION.md adapter."""
    import ctypes as C
    rt = _runtime()
    m, y0 = cases.ccw()
    g, o = rt.RhsHandle(m), oracle_mod.OracleRhs(m, 0)
    g.set_step_inputs(); o.set_step_inputs()
    dy = np.zeros(m.num_y)
    rc = rt.lib().shud_rhs_cvrhs(0.0, y0.ctypes.data, dy.ctypes.data, g.h)
    assert rc == 0
    assert_close(dy, o.eval(0.0, y0)[0], what="cvrhs")


@pytest.mark.parametrize("kind", ["et_negative", "effkh", "nan"])
def test_error_paths(kind, oracle_mod, layout):
    """Where the reference would myexit(), the GPU reports the same exit code and element."""
    rt = _runtime()
    m, y0 = cases.ccw()
    y = y0.copy()
    if kind == "et_negative":
        m.step["pot_evap"][[700, 300]] = -1e-3          # CheckNonNegative(Es) -> exit 10
        m.step["lai"][:] = 0.0
        y[300] = 0.01
        y[700] = 0.01
    elif kind == "effkh":
        m.par["macKsatH"][[900, 400]] = 1e15           # effKH > 1e9 -> exit 13
        aq = m.par["aquifer_depth"]
        for i in (900, 400):
            y[2 * m.num_ele + i] = aq[i] - 0.5 * m.par["macD"][i]
    else:
        y[2 * m.num_ele + 500] = np.nan                 # NaN groundwater -> CheckNANij -> exit 10
    g, o = rt.RhsHandle(m), oracle_mod.OracleRhs(m, 0)
    g.set_step_inputs(); o.set_step_inputs()
    _, code, idx, _ = o.eval(0.0, y)
    assert code in (10, 13)
    with pytest.raises(rt.ShudRhsError) as ei:
        g.eval(0.0, y)
    e = ei.value.err
    assert e["exit_code"] == code
    fi = e["first_index"]
    if kind == "et_negative":
        assert min(v for v in (fi[2], fi[3]) if v >= 0) == idx
    elif kind == "effkh":
        assert fi[1] == idx
    else:
        assert fi[0] == idx


def test_lake_without_bathymetry_rejected():
    rt = _runtime()
    m, _ = cases.ccw()
    m.ilake = np.zeros(m.num_ele, dtype=np.int32)
    m.ilake[5] = 1                                   # a lake element but num_lake = 0
    with pytest.raises(rt.ShudRhsError) as ei:
        rt.RhsHandle(m)
    assert ei.value.code == abi.SHUD_ERR_ARG


@pytest.mark.parametrize("case", ["qhh", "qhh_variant"])
def test_lakes(case, oracle_mod):
    """Lake module: qhh (688 lake elements, bank edges) and reaches redirected into the lake;
    IC state, a low and a high lake stage, 3 stateful calls each, every diagnostic incl. the lake sums."""
    m, y = getattr(cases, case)()
    ys = [y.copy(), workload.random_state(m, seed=31)]
    ys[1][-1] = 300.0                                 # lake level above its banks: weir exchange both ways
    _compare_sequence(m, ys, abi.SHUD_MODE_SERIAL, oracle_mod, label=case, layout="packed")


def test_lakes_unsupported_modes(monkeypatch):
    rt = _runtime()
    m, _ = cases.qhh()
    with pytest.raises(rt.ShudRhsError) as ei:
        rt.RhsHandle(m, mode=abi.SHUD_MODE_OMP)       # the OMP path has no lake physics
    assert ei.value.code == abi.SHUD_ERR_UNSUPPORTED
    monkeypatch.setenv("SHUD_RHS_PACKED", "0")
    with pytest.raises(rt.ShudRhsError) as ei:
        rt.RhsHandle(m)                               # lakes need the packed layout
    assert ei.value.code == abi.SHUD_ERR_UNSUPPORTED


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_syn_1m(mode, oracle_mod, layout):
    """syn-1M: full-size parity against the oracle, 2 successive calls."""
    from shud_rhs import synth
    m = synth.synth_model(1_000_000)
    m.step = workload.random_step_inputs(m)
    y = workload.random_state(m)
    _compare_sequence(m, [y], mode, oracle_mod, ncalls=2, diag=False, label="syn-1M", layout=layout)


def test_fu_nonunit_and_packed_flags(oracle_mod):
    """fu_Surf / fu_Sub != 1 (cryosphere on) switches the packed kernel to reading them; back to 1 -> skip."""
    rt = _runtime()
    m, y0 = cases.ccw()
    g, o = rt.RhsHandle(m), oracle_mod.OracleRhs(m, 0)
    g.set_step_inputs(); o.set_step_inputs()
    rng = np.random.default_rng(4)
    for fu in [rng.uniform(0.2, 1.0, m.num_ele), np.ones(m.num_ele)]:
        st = {"fu_surf": fu, "fu_sub": fu[::-1].copy()}
        g.set_step_inputs(st); o.set_step_inputs(st)
        for c in range(2):
            assert_close(g.eval(0.0, y0), o.eval(0.0, y0)[0], what="fu step")


def test_syn_10m(oracle_mod):
    """syn-10M (BASELINE configs[4]'s mesh, the bench workload) on one GPU against the oracle at the strict
    tolerance: serial semantics, the packed layout the bench runs, 2 successive calls (carried state)."""
    from shud_rhs import synth
    m = synth.synth_model(10_000_000)
    m.step = workload.random_step_inputs(m)
    y = workload.random_state(m)
    _compare_sequence(m, [y], abi.SHUD_MODE_SERIAL, oracle_mod, ncalls=2, diag=False, label="syn-10M",
                      layout="packed")


@pytest.mark.parametrize("kind", ["hybrid1", "hybrid", "l2", "soa"])
def test_many_classes(oracle_mod, monkeypatch, kind):
    """Per-element calibrated parameters: > 128 distinct parameter tuples.  Default: the hybrid layout (KsatH and Sy
    streamed per element, the rest in the LDS class table); with SHUD_RHS_HYB=0 the SoA kernel, or with
    SHUD_RHS_L2_CLASS=1 the packed kernel reading its class table from L2 (record-major, no LDS copy)."""
    if not kind.startswith("hybrid"):
        monkeypatch.setenv("SHUD_RHS_HYB", "0")
        monkeypatch.setenv("SHUD_RHS_L2_CLASS", "1" if kind == "l2" else "0")
    m, y = cases.variant(20000, seed=17)
    m.par["KsatH"] = m.par["KsatH"] * (1.0 + 1e-7 * (np.arange(m.num_ele) % 300))
    if kind != "hybrid1":                        # hybrid1: KsatH alone (one streamed field, the 8-B record)
        m.par["Sy"] = m.par["Sy"] * (1.0 + 1e-9 * (np.arange(m.num_ele) % 7))
    if kind.startswith("hybrid"):
        lay = _runtime().RhsHandle(m).layout()
        assert lay["packed"] and lay.get("streamed_fields") == (1 if kind == "hybrid1" else 2), lay
        assert lay["n_classes"] <= 128, lay
    for mode in (abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP):
        _compare_sequence(m, [y] + cases.states(m, None, 1, seed=3), mode, oracle_mod, ncalls=2,
                          label=f"many-class {kind}", layout="soa" if kind == "soa" else "packed")


def _class_count(m):
    """distinct parameter tuples of a model (the packed layout's classes: shud_rhs.cpp build_packed)"""
    keys = ["macD", "macKsatH", "geo_vAreaF", "KsatH", "KsatV", "infKsatV", "hAreaF", "macKsatV", "ThetaS", "ThetaR",
            "Beta", "infD", "Sy", "RzD", "VegFrac", "ImpAF"]
    cols = [np.asarray(m.par[k], np.float64) for k in keys] + [np.asarray(m.ele["depression"], np.float64),
                                                               np.asarray(m.ele["rough"], np.float64)]
    return np.unique(np.stack(cols, 1), axis=0).shape[0]


@pytest.mark.parametrize("target", ["mid", "max"])
def test_lds_big_class_table(oracle_mod, monkeypatch, target):
    """129..560 parameter classes with the hybrid layout off (SHUD_RHS_HYB=0): the 1024-thread workgroups that stage
    the whole class table + pow tables in LDS (shud_ele_kernel_packed_big), serial and OMP, against the oracle.
    "max" sits at the LDS bound (kLdsClassMaxBig = 560 classes: the dynamic-LDS attribute and the 16-B table copy at
    their largest)."""
    monkeypatch.setenv("SHUD_RHS_HYB", "0")
    m, y = cases.variant(20000, seed=29)
    base, k = m.par["KsatH"].copy(), np.arange(m.num_ele)
    mult, n = 12, 0
    for mm in ([12] if target == "mid" else range(12, 40)):    # "max": the most classes still <= 560
        m.par["KsatH"] = base * (1.0 + 1e-7 * (k % mm))
        nn = _class_count(m)
        if nn > 560:
            break
        mult, n = mm, nn
    m.par["KsatH"] = base * (1.0 + 1e-7 * (k % mult))
    assert 128 < n <= 560 and (target == "mid" or n > 520), (mult, n)
    lay = _runtime().RhsHandle(m).layout()
    assert lay["packed"] and not lay.get("streamed_fields") and lay["n_classes"] == n, lay
    for mode in (abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP):
        _compare_sequence(m, [y] + cases.states(m, None, 1, seed=7), mode, oracle_mod, ncalls=2,
                          label=f"big class table {n}", layout="packed")


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_mid_class_count(mode, oracle_mod):
    """~66 parameter classes: the LDS class table without the DY-tail LDS slots (they fit beside tables of up to
    ~35 classes only, shud_ele_packed.hip LSP), against the oracle."""
    m, y = cases.variant(20000, seed=23)
    m.par["KsatH"] = m.par["KsatH"] * (1.0 + 1e-7 * (np.arange(m.num_ele) % 2))
    lay = _runtime().RhsHandle(m, mode=mode).layout()
    assert lay["packed"] and not lay.get("streamed_fields") and 40 <= lay["n_classes"] <= 128, lay
    _compare_sequence(m, [y] + cases.states(m, None, 1, seed=5), mode, oracle_mod, ncalls=2, label="mid-class",
                      layout="packed")


def _hybrid_model(n=20000, seed=19):
    """every element its own KsatH, Rough, macD and Sy (four streamed fields, the 32-B per-element record)"""
    m, y = cases.variant(n, seed=seed)
    k = np.arange(m.num_ele)
    m.par["KsatH"] = m.par["KsatH"] * (1.0 + 1e-6 * k / m.num_ele)
    m.par["macD"] = m.par["macD"] * (1.0 + 1e-3 * ((k * 7) % 11))
    m.par["Sy"] = m.par["Sy"] * (1.0 + 1e-9 * (k % 13))
    rough = m.ele["rough"] * (1.0 + 1e-2 * ((k * 3) % 5))
    m.ele["rough"] = rough
    nb = m.nabr.reshape(3, -1)          # avgRough = (Rough_i + Rough_j) / 2 (Element.cpp:253), own Rough on a boundary
    m.ele["avg_rough"] = np.where(nb >= 0, 0.5 * (rough[None, :] + rough[np.maximum(nb, 0)]),
                                  rough[None, :]).reshape(-1)
    return m, y


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_hybrid_layout(mode, oracle_mod):
    """The hybrid layout with four streamed fields, each per-element unique or nearly (KsatH, macD, Sy, Rough: the
    neighbour's streamed KsatH / macD / Rough enter the edge fluxes), against the oracle, 3 stateful calls on 3
    states, every diagnostic."""
    m, y = _hybrid_model()
    lay = _runtime().RhsHandle(m, mode=mode).layout()
    assert lay["packed"] and lay.get("streamed_fields") == 4, lay
    _compare_sequence(m, [y] + cases.states(m, None, 2, seed=41), mode, oracle_mod, label="hybrid", layout="packed")


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_edge_meshes(mode, oracle_mod, layout):
    """Edge cases of the mesh: no rivers at all (NR = NS = 0, empty river launch), the smallest synthetic meshes
    (8 and 48 elements, every element on or next to the boundary), and a single triangle whose three edges are
    all open boundaries."""
    from shud_rhs import synth
    cases_ = [("riverless ccw",) + cases.riverless(), ("single open", *cases.single_element(0)),
              ("single closed", *cases.single_element(1))]
    for n in (2, 50):
        m = synth.synth_model(n)
        m.step = workload.random_step_inputs(m, seed=n)
        cases_.append((f"synth {m.num_ele}", m, workload.random_state(m, seed=n)))
    for label, m, y in cases_:
        _compare_sequence(m, [y] + cases.states(m, None, 2, seed=31), mode, oracle_mod, ncalls=2, label=label,
                          layout=layout)
