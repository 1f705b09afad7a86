import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shud-up_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")
ORACLE_DIR = os.path.join(ROOT, "oracle")
PKG_DIR = os.path.join(ROOT, "shud-up_amd")

# GPU parity tolerance: |gpu - ref| <= RTOL*|ref| + ATOL per state.
RTOL = 1e-12
ATOL = 1e-15


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def load_fixture(name):
    from shud_rhs import ShudModel
    m = ShudModel.load(os.path.join(GOLDEN, f"{name}_model.npz"))
    y0 = np.load(os.path.join(GOLDEN, f"{name}_y0.npy"))
    return m, y0


def assert_close(got, ref, rtol=RTOL, atol=ATOL, what=""):
    got = np.asarray(got)
    ref = np.asarray(ref)
    both_nan = np.isnan(got) & np.isnan(ref)
    err = np.abs(got - ref)
    bad = ~((err <= rtol * np.abs(ref) + atol) | both_nan | (got == ref))
    if bad.any():
        i = np.nonzero(bad)[0][:5]
        raise AssertionError(f"{what}: {bad.sum()} of {bad.size} entries outside tolerance; first {i}: "
                             f"got {got[i]} ref {ref[i]}")
    finite = np.isfinite(ref) & (ref != 0)
    rel = (err[finite] / np.abs(ref[finite])).max() if finite.any() else 0.0
    return float(err[~both_nan].max() if (~both_nan).any() else 0.0), float(rel)


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    return oracle
