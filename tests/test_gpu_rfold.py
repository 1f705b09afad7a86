"""River fold (shud_ele_packed.hip shud_rhs_kernel_packed_rf): the elements, the QrivDown pre-pass
and the reaches in ONE launch, the reach tiles starting once the element tiles and QrivDown blocks they read have
published their write-through results.  Same arithmetic as the element + river launches, so every DY word must equal
the two-launch path's (SHUD_RHS_RFOLD=0), including under a late element tile (the hand-off tested under uneven load,
MI355X guide Guideline 16), and a tile that never publishes must end in the fatal SHUD_EF_HALO_WAIT."""
import numpy as np
import pytest

import cases
from shud_rhs import abi, workload

pytestmark = pytest.mark.gpu


def _handles(m, mode, monkeypatch):
    from shud_rhs import runtime as rt
    monkeypatch.setenv("SHUD_RHS_RFOLD", "1")
    f = rt.RhsHandle(m, mode=mode)
    monkeypatch.setenv("SHUD_RHS_RFOLD", "0")
    two = rt.RhsHandle(m, mode=mode)
    monkeypatch.delenv("SHUD_RHS_RFOLD")
    assert f.layout().get("river_fold") and not two.layout().get("river_fold"), (f.layout(), two.layout())
    f.set_step_inputs()
    two.set_step_inputs()
    return f, two


def _same(a, b):
    return np.array_equal(a, b, equal_nan=True)


def _junctions():
    import test_gpu_parity
    return test_gpu_parity._junction_model()


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
@pytest.mark.parametrize("case", ["ccw", "heihe", "variant", "junctions", "syn1m"])
def test_river_fold_bit_identical(case, mode, monkeypatch):
    """Folded vs two launches on the reference's basins, the branch-variant mesh (outlets, +-BC reaches, bank slopes),
    the junction shapes (0..14 upstream reaches) and syn-1M: 3 states x 2 stateful calls, every DY word."""
    from shud_rhs import synth
    if case == "ccw":
        m, y0 = cases.ccw()
    elif case == "heihe":
        m, y0 = cases.heihe()
    elif case == "variant":
        m, y0 = cases.variant(20000, seed=13)
    elif case == "junctions":
        m, y0 = _junctions()
    else:
        m = synth.synth_model(1_000_000)
        m.step = workload.random_step_inputs(m)
        y0 = workload.random_state(m)
    f, two = _handles(m, mode, monkeypatch)
    try:
        states = ([y0] if y0 is not None else []) + cases.states(m, None, 2, seed=61)
        for si, y in enumerate(states):
            for c in range(2):
                a, b = f.eval(0.0, y), two.eval(0.0, y)
                assert _same(a, b), f"{case} state {si} call {c}: {(~((a == b) | (np.isnan(a) & np.isnan(b)))).sum()} differ"
        assert f.get_error()["flags"] == two.get_error()["flags"]
    finally:
        f.close()
        two.close()


@pytest.mark.parametrize("mode", [abi.SHUD_MODE_SERIAL, abi.SHUD_MODE_OMP])
def test_river_fold_late_tile(mode, monkeypatch):
    """A genuinely late element tile: the tile the most reach tiles depend on spins 300 us before computing, so those
    reach tiles poll its flag while the rest of the launch runs; a new state on every call (the segment fluxes change
    each eval, so a stale line would show); every DY word equals the two-launch path's."""
    from shud_rhs import synth
    m = synth.synth_model(400_000)
    m.step = workload.random_step_inputs(m)
    f, two = _handles(m, mode, monkeypatch)
    try:
        tile = f.debug_rfold(-1, spin_us=300.0)
        assert tile >= 0
        yb, db = f.device_alloc(8 * m.num_y), f.device_alloc(8 * m.num_y)
        try:
            for call in range(6):
                y = workload.random_state(m, seed=200 + call)
                f.h2d(yb, y)
                f.eval_device(0.0, yb, db)
                got = f.d2h(np.zeros(m.num_y), db)
                want = two.eval(0.0, y)
                e = f.get_error()
                assert e["flags"] & 0x80 == 0, f"call {call}: SHUD_EF_HALO_WAIT"
                assert _same(got, want), f"call {call}: {(~((got == want) | (np.isnan(got) & np.isnan(want)))).sum()} differ"
        finally:
            f.device_free(yb)
            f.device_free(db)
    finally:
        f.close()
        two.close()


def test_river_fold_tile_never_publishes(monkeypatch):
    """A tile that spins past the reach tiles' poll bound: their bounded poll ends in the fatal SHUD_EF_HALO_WAIT and
    the host eval returns an error; disarmed, the next evals are bit-identical to the two-launch path again."""
    from shud_rhs import synth
    m = synth.synth_model(100_000)
    m.step = workload.random_step_inputs(m)
    y = workload.random_state(m, seed=7)
    f, two = _handles(m, abi.SHUD_MODE_SERIAL, monkeypatch)
    try:
        f.debug_rfold(-1, spin_us=200_000.0, timeout_ms=10.0)
        with pytest.raises(RuntimeError):
            f.eval(0.0, y)
        assert f.get_error()["flags"] & 0x80
        f.debug_rfold(-1, spin_us=0.0, timeout_ms=5000.0)
        f.clear_error()
        f.set_step_inputs()
        two.set_step_inputs()
        for c in range(2):
            a, b = f.eval(0.0, y), two.eval(0.0, y)
            assert _same(a, b), f"call {c} after disarming"
        assert f.get_error()["flags"] & 0x80 == 0
    finally:
        f.close()
        two.close()
