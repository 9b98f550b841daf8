"""The library's Sobol candidate generator (kind BO_CAND_SOBOL) against scipy.stats.qmc.Sobol
(scramble=False), the generator BASELINE configs C4/C5 name: direction numbers and points
bit-identical.  Host entry points only (no device): the device generator evaluates the same
bo_sobol_coord on the same direction numbers (tests/test_gpu_configs.py checks the device side)."""

import ctypes

import numpy as np
import pytest

qmc = pytest.importorskip("scipy.stats.qmc")


@pytest.fixture(scope="module")
def lib():
    from bayesopt_smart_amd import _lib
    return _lib.load()


@pytest.mark.parametrize("dim", range(1, 9))
def test_direction_numbers_match_scipy(lib, dim):
    for bits in (30, 32, 20):
        out = np.empty((dim, bits), dtype=np.uint32)
        assert lib.bo_sobol_direction_numbers(dim, bits, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))) == 0
        ref = qmc.Sobol(dim, scramble=False, bits=bits)._sv[:, :bits]
        np.testing.assert_array_equal(out, ref.astype(np.uint32))


@pytest.mark.parametrize("dim", [1, 2, 5, 6, 8])
def test_points_match_scipy_bit_exact(dim):
    from bayesopt_smart_amd.predict import CandidateSet
    m = 1 << 13
    cs = CandidateSet.sobol_set(dim, m, scale=300.0)
    got = cs.points(np.arange(m))
    ref = qmc.Sobol(dim, scramble=False).random(m) * 300.0
    np.testing.assert_array_equal(got, ref)
    # an affine box (scipy's qmc.scale: lo + sample * (hi - lo))
    lo, hi = np.arange(dim) - 7.5, np.arange(dim) * 3.0 + 11.0
    cs = CandidateSet.sobol_set(dim, m, lo=lo, scale=hi - lo)
    np.testing.assert_array_equal(cs.points(np.arange(m)),
                                  qmc.scale(qmc.Sobol(dim, scramble=False).random(m), lo, hi))


def test_points_random_access_deep_indices():
    """Points far into the sequence (C5's 2^22 set), computed from the index alone."""
    from bayesopt_smart_amd.predict import CandidateSet
    m = 1 << 22
    cs = CandidateSet.sobol_set(6, m, scale=300.0)
    ref = qmc.Sobol(6, scramble=False).random(m) * 300.0
    idx = np.random.default_rng(0).choice(m, 5000, replace=False)
    np.testing.assert_array_equal(cs.points(idx), ref[idx])
    with pytest.raises(Exception):
        cs.points(np.array([1 << 30]))                   # beyond 2^bits
