import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_golden(name):
    path = os.path.join(GOLDEN, f"{name}.npz")
    if not os.path.exists(path):
        pytest.skip(f"golden fixture {name} not generated")
    return np.load(path, allow_pickle=False)


@pytest.fixture
def golden():
    return load_golden


def kinv_of(d):
    """K^-1 of a predict fixture: stored (small N) or recomputed with the oracle and pinned
    to the reference's bytes by the stored sha256 digest (large N)."""
    import hashlib
    from oracle import oracle_np as O
    if "Kinv" in d.files if hasattr(d, "files") else "Kinv" in d:
        return d["Kinv"]
    n = d["x"].shape[0]
    km = np.zeros((d["pm"].shape[0], n, n))
    O.update_k(km, d["x"], 0, n, d["pv"], d["ls"])
    kinv = O.invert_k(n, km)
    # the Gram is pinned bit-for-bit; LAPACK's inverse is host-dependent (OpenBLAS picks its
    # kernels per CPU), so K^-1 is only bit-equal on the host that generated the fixture
    assert hashlib.sha256(km.tobytes()).digest() == bytes(d["K_sha256"])
    return kinv


class Fixture(dict):
    """dict view of a predict fixture with Kinv always present."""


def predict_fixture(name):
    d = load_golden(name)
    f = Fixture({k: d[k] for k in d.files})
    f["Kinv"] = kinv_of(d)
    return f
