import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: full-size BASELINE configurations")


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(GOLDEN, "golden_small.npz"))


@pytest.fixture(scope="session")
def golden_full():
    import json
    with open(os.path.join(GOLDEN, "golden_full.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


def snr_close(a, b, rtol=1e-4):
    """BASELINE.json tolerance for S/N: 1e-4 relative.  S/N is in units of the
    noise sigma, so the relative scale is max(|ref|, 1): a value of 0.003 sigma
    is compared to 1e-4 sigma, not to 3e-7."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        return False, f"shape {a.shape} vs {b.shape}"
    err = np.abs(a - b) / np.maximum(np.abs(b), 1.0)
    worst = float(err.max()) if err.size else 0.0
    return worst <= rtol, f"max scaled err {worst:.3e}"
