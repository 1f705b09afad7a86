"""GPU: randomized property tests (hypothesis) — drawn meshes, states, step inputs and integrator
problems through the HIP path, each property checked against the CPU restatement or against the GPU itself:

  * RHS parity on random branch-variant meshes (size, seed, serial/OMP, open/closed boundary, both device
    layouts, successive stateful calls): the conftest tolerance 1e-12 |ref| + 1e-15 per entry,
  * run-to-run determinism: two fresh handles on the same inputs give bit-identical DY and diagnostics,
  * the device integrator on the n-component decay problem with random n (one partial block up to many
    reduction blocks, odd tails), tolerances and initial step: every output and counter bit-identical to the
    oracle with its reductions in the device's block order (the vector kernels' grid shapes differ per n).
Examples are few and small so the file runs in well under a minute."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import cases
from conftest import assert_close
from shud_rhs import abi, workload

pytestmark = pytest.mark.gpu

SETTINGS = settings(max_examples=12, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


@SETTINGS
@given(n=st.integers(200, 5000), seed=st.integers(0, 10_000), mode=st.sampled_from([0, 1]),
       open_boundary=st.booleans(), packed=st.sampled_from(["1", "0"]), calls=st.integers(1, 3))
def test_random_meshes_vs_oracle(n, seed, mode, open_boundary, packed, calls, monkeypatch):
    import oracle
    from shud_rhs import runtime as rt
    monkeypatch.setenv("SHUD_RHS_PACKED", packed)
    m, y = cases.variant(n, seed=seed)
    m.close_boundary = 0 if open_boundary else 1
    m.step = workload.random_step_inputs(m, seed=seed + 7)
    g, o = rt.RhsHandle(m, mode=mode), oracle.OracleRhs(m, mode)
    try:
        g.set_step_inputs()
        o.set_step_inputs()
        for si, yy in enumerate((y, workload.random_state(m, seed=seed + 1))):
            for c in range(calls):
                ref, code, _, _ = o.eval(0.0, yy)
                assert code == 0
                assert_close(g.eval(0.0, yy), ref, what=f"n={n} seed={seed} state {si} call {c}")
    finally:
        g.close()


@SETTINGS
@given(n=st.integers(200, 20000), seed=st.integers(0, 10_000), mode=st.sampled_from([0, 1]))
def test_run_to_run_determinism(n, seed, mode):
    from shud_rhs import runtime as rt
    m, y = cases.variant(n, seed=seed)
    out = []
    for _ in range(2):
        g = rt.RhsHandle(m, mode=mode)
        try:
            g.set_step_inputs()
            a = g.eval(0.0, y)
            b = g.eval(0.0, y)                     # the stateful second call as well
            out.append((a, b, g.diagnostics()))
        finally:
            g.close()
    (a0, b0, d0), (a1, b1, d1) = out
    assert np.array_equal(a0, a1, equal_nan=True) and np.array_equal(b0, b1, equal_nan=True)
    for k in abi.FLUXOUT_ORDER:
        assert np.array_equal(d0[k], d1[k], equal_nan=True), k


# the CPU restatement integrates sequentially: sizes just past the 2048-block reduction grid exercise the
# grid-stride tail without spending minutes in the oracle (12 examples up to 2600 blocks took 133 s, 8 up to 2100
# blocks 83 s; 5 keep both size bands under derandomize)
@settings(max_examples=5, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(blocks=st.one_of(st.integers(0, 300), st.integers(2044, 2100)), tail=st.integers(1, 255),
       rtol_e=st.integers(4, 8), atol_e=st.integers(8, 12), h0_e=st.integers(2, 6))
def test_integrator_random_sizes_bit_identical(blocks, tail, rtol_e, atol_e, h0_e):
    """decayn with n = 256*blocks + tail: the reduction grid (min(ceil(n/256), 2048) blocks, grid-stride:
    above 2048 blocks each thread sums several entries) and the element-wise grid (one entry per thread) both
    see partial blocks and odd tails."""
    import ctypes as C
    import os

    import oracle
    from conftest import PKG_DIR
    from shud_rhs import runtime as rt
    kat = C.CDLL(os.path.join(PKG_DIR, "libshud_kat.so"))
    kat.shud_kat_ode_user.restype = C.c_void_p
    kat.shud_kat_ode_user.argtypes = [C.c_int]
    kat.shud_kat_ode_stream.restype = C.c_void_p
    kat.shud_kat_ode_stream.argtypes = [C.c_void_p]
    kat.shud_kat_ode_set_n.argtypes = [C.c_int64]
    kat.shud_kat_ode_free.argtypes = [C.c_void_p]
    rt.lib()
    n = 256 * blocks + tail
    rtol, atol, h0 = 10.0 ** -rtol_e, 10.0 ** -atol_e, 10.0 ** -h0_e
    y0 = 1.0 + 0.5 * np.sin(np.arange(n))
    u = kat.shud_kat_ode_user(3)
    kat.shud_kat_ode_set_n(n)
    fn = (C.cast(kat.shud_kat_ode_rhs, C.c_void_p).value, u, kat.shud_kat_ode_stream(u))
    oracle.OracleOde.set_reduction_order(1)
    d = o = None
    try:
        d = rt.OdeSolver(None, 0.0, y0, rtol, atol, h0, 0.0, 0.0, fn=fn)
        o = oracle.OracleOde("decayn", 0.0, y0, rtol, atol, h0, 0.0, 0.0)
        for tout in (0.01, 0.5, 3.0):
            fd, td, yd = d.solve(tout)
            fo, to, yo = o.solve(tout)
            assert (fd, td) == (fo, to)
            assert np.array_equal(yd, yo), f"n={n}: {(yd != yo).sum()} entries differ at t={tout}"
        sd, so = d.stats(), o.stats()
        for k in ("nst", "nfe", "nni", "nli", "netf", "ncfn", "qcur", "hcur"):
            assert sd[k] == so[k], (k, sd[k], so[k])
    finally:
        oracle.OracleOde.set_reduction_order(0)
        if d is not None:
            d.close()
        kat.shud_kat_ode_free(C.c_void_p(u))
