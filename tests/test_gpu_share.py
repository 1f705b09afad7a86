"""In-tile edge sharing (shud_ele_packed.hip SH, the host's assignment in shud_rhs.cpp build_packed): an interior edge
evaluated by one element and read, sign-corrected, by the other must leave every DY word and every error word exactly
as evaluating the edge from both sides does (SHUD_RHS_SHARE=0), and agree with the oracle.  The states aim at the
sign rules: equal surface / groundwater heads across edges (dh == +0, dhg == +0: no negation), dry cells (no Manning),
the groundwater zero branches, negative states (the OMP clamps), NaN and infinite heads (the receiver evaluates the
edge itself, and the error exit names the same element)."""
import numpy as np
import pytest

import cases
from conftest import assert_close
from shud_rhs import abi, synth, workload

pytestmark = pytest.mark.gpu


def _rt():
    from shud_rhs import runtime
    return runtime


def _handles(m, mode, monkeypatch):
    rt = _rt()
    monkeypatch.setenv("SHUD_RHS_SHARE", "1")
    a = rt.RhsHandle(m, mode=mode)
    monkeypatch.setenv("SHUD_RHS_SHARE", "0")
    b = rt.RhsHandle(m, mode=mode)
    monkeypatch.delenv("SHUD_RHS_SHARE")
    la, lb = a.layout(), b.layout()
    assert la["packed"] and la.get("shared_edges", 0) > 0.3 * m.num_ele, la
    assert "shared_edges" not in lb, lb
    a.set_step_inputs()
    b.set_step_inputs()
    return a, b


def _run(h, y):
    rt = _rt()
    try:
        return h.eval(0.0, y), None
    except rt.ShudRhsError as e:
        err = dict(e.err)
        err.pop("message", None)
        h.clear_error()
        return None, err


def _same_bits(a, b, what):
    assert a.shape == b.shape
    ua, ub = a.view(np.uint64), b.view(np.uint64)
    bad = np.nonzero(ua != ub)[0]
    assert bad.size == 0, f"{what}: {bad.size} words differ, first {bad[:5]}: {a[bad[:5]]} vs {b[bad[:5]]}"


def _states(m, seed):
    """random states plus the sign-rule cases, each on a random half of the elements"""
    NE = m.num_ele
    rng = np.random.default_rng(seed)
    zs, zb = np.asarray(m.ele["z_surf"]), np.asarray(m.ele["z_bottom"])
    out = [workload.random_state(m, seed=seed)]
    y = workload.random_state(m, seed=seed + 1)
    half = rng.random(NE) < 0.5
    H = float(np.max(zs)) + 0.25                     # zs/2 <= H <= 2 zs: H - zs and (H - zs) + zs exact
    Hg = float(np.max(zb)) + 5.0
    y[:NE][half] = H - zs[half]                       # equal surface heads: dh == +0 across such edges
    y[2 * NE:3 * NE][half] = Hg - zb[half]            # equal groundwater heads: dhg == +0
    out.append(y)
    y = workload.random_state(m, seed=seed + 2)
    y[:NE][rng.random(NE) < 0.5] = 0.0                # dry cells: ym = 0, no Manning
    low = rng.random(NE) < 0.4
    y[2 * NE:3 * NE][low] = rng.uniform(0.0, 0.02, low.sum())   # the groundwater zero branches
    out.append(y)
    y = workload.random_state(m, seed=seed + 3)
    neg = rng.random(NE) < 0.3
    y[:NE][neg] = -rng.uniform(0.0, 0.1, neg.sum())   # negative surface (MODE 1 clamps it)
    out.append(y)
    return out


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
@pytest.mark.parametrize("mesh", ["syn", "variant"])
def test_share_same_bits_and_oracle(mesh, mode, oracle_mod, monkeypatch):
    """syn (closed boundary, fu = 1) and the branch-variant mesh (open boundary, BC elements, SS flags, fu != 1):
    sharing on vs off bit for bit over stateful call sequences, and both against the oracle"""
    if mesh == "syn":
        m = synth.synth_model(20000, seed=41)
        m.step = workload.random_step_inputs(m, seed=3)
    else:
        m, _ = cases.variant(20000, seed=43)
    a, b = _handles(m, mode, monkeypatch)
    o = oracle_mod.OracleRhs(m, mode)
    o.set_step_inputs()
    for si, y in enumerate(_states(m, 70)):
        for c in range(2):
            ga, ea = _run(a, y)
            gb, eb = _run(b, y)
            ref, code, _, _ = o.eval(0.0, y)
            assert ea is None and eb is None and code == 0, (ea, eb, code)
            _same_bits(ga, gb, f"{mesh} state {si} call {c}")
            assert_close(ga, ref, what=f"{mesh} shared, state {si} call {c}")
    a.close()
    b.close()


@pytest.mark.parametrize("kind", ["nan_surface", "nan_gw", "inf_surface"])
def test_share_nonfinite_heads(kind, oracle_mod, monkeypatch):
    """A NaN or infinite head on a shared edge: the receiver evaluates the edge itself (or sees the publisher's
    non-finite flux), so the error exit and its first element are those of the unshared kernel and the oracle"""
    m = synth.synth_model(20000, seed=41)
    m.step = workload.random_step_inputs(m, seed=3)
    a, b = _handles(m, abi.SHUD_MODE_SERIAL, monkeypatch)
    o = oracle_mod.OracleRhs(m, 0)
    o.set_step_inputs()
    NE = m.num_ele
    y = workload.random_state(m, seed=5)
    rng = np.random.default_rng(9)
    k = rng.choice(NE, 6, replace=False)
    if kind == "nan_surface":
        y[k] = np.nan
    elif kind == "nan_gw":
        y[2 * NE + k] = np.nan
    else:
        y[k] = np.inf
        y[k[:3] + 1] = np.inf                          # neighbours both infinite: inf - inf = NaN head difference
    ga, ea = _run(a, y)
    gb, eb = _run(b, y)
    _, code, idx, ekind = o.eval(0.0, y)
    assert ea == eb, (ea, eb)
    if code:
        assert ea is not None and ea["exit_code"] == code
        if ekind == abi.EF_NAN_QELE:                          # CheckNANij: the first element with a NaN lateral flux
            assert ea["first_index"][0] == idx, (ea["first_index"], idx)
    else:
        _same_bits(ga, gb, kind)
    a.close()
    b.close()


def test_share_counts_real_meshes(monkeypatch):
    """the reference's own meshes: how many edges the assignment shares (their numbering is not tile-local), and
    the same bits either way"""
    for name in ("ccw", "heihe"):
        m, y0 = getattr(cases, name)()
        rt = _rt()
        monkeypatch.setenv("SHUD_RHS_SHARE", "1")
        a = rt.RhsHandle(m)
        monkeypatch.setenv("SHUD_RHS_SHARE", "0")
        b = rt.RhsHandle(m)
        monkeypatch.delenv("SHUD_RHS_SHARE")
        a.set_step_inputs()
        b.set_step_inputs()
        for y in cases.states(m, y0, 2):
            _same_bits(a.eval(0.0, y), b.eval(0.0, y), name)
        print(name, m.num_ele, a.layout())
        a.close()
        b.close()


from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=10, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(n=st.integers(2000, 30000), seed=st.integers(0, 10_000), mode=st.sampled_from([0, 1]),
       open_boundary=st.booleans())
def test_share_random_meshes(n, seed, mode, open_boundary, monkeypatch):
    """drawn branch-variant meshes (sizes that end in a partial tile, either boundary kind, both modes): sharing on
    vs off bit for bit, for a random state and the equal-head / dry-cell states"""
    m, _ = cases.variant(n, seed=seed)
    m.close_boundary = 0 if open_boundary else 1
    m.step = workload.random_step_inputs(m, seed=seed + 7)
    a, b = _handles(m, mode, monkeypatch)
    try:
        for si, y in enumerate(_states(m, seed)[:3]):
            ga, ea = _run(a, y)
            gb, eb = _run(b, y)
            assert ea == eb, (ea, eb)
            if ea is None:
                _same_bits(ga, gb, f"n={n} seed={seed} state {si}")
    finally:
        a.close()
        b.close()
