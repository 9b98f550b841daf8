"""Pin the CPU oracle (oracle/oracle_np.py) against vectors produced by the reference itself.

The fixtures come from tests/golden/make_golden.py (reference imported in its debug
mode).  Where the arithmetic order is the same the oracle must match bit-for-bit;
the exp/LAPACK-dependent outputs are allowed 1-ulp-class differences.
"""
import os

import numpy as np
import pytest

from oracle import oracle_np as O
from conftest import kinv_of, predict_fixture


def _chain(d, with_kinv=True):
    x, y, cand = d["x"], d["y"], d["cand"]
    kinv = kinv_of(d) if with_kinv else None
    return O.predict_acquire(x, y, cand, d["pm"], d["pv"], d["ls"], d["betas"], kinv=kinv, chunk=4096)


@pytest.mark.parametrize("name", ["g1_predict_2d", "g1_grid", "g2_predict_512", "g3_predict_6d3o", "g7_illcond"])
def test_gram_and_inverse(golden, name):
    d = golden(name)
    n = d["x"].shape[0]
    if "K" not in d.files:
        import hashlib
        kinv = kinv_of(d)   # recomputes the Gram and checks its sha256 against the reference's
        if os.path.exists("/root/reference"):   # the fixture's host: LAPACK inverse bit-equal too
            assert hashlib.sha256(kinv.tobytes()).digest() == bytes(d["Kinv_sha256"])
        return
    km = np.zeros((d["K"].shape[0], n, n))
    O.update_k(km, d["x"], 0, n, d["pv"], d["ls"])
    np.testing.assert_array_equal(km, d["K"])
    kinv = O.invert_k(n, km)
    np.testing.assert_array_equal(kinv, d["Kinv"])


def test_kstar_bitexact(golden):
    d = golden("g1_predict_2d")
    ks_ref = d["kstar_head"]
    n = d["x"].shape[0]
    ks = np.zeros((2, n, ks_ref.shape[2]))
    O.update_k_star(ks, d["x"], d["cand"][: ks_ref.shape[2]], 0, n, d["pv"], d["ls"])
    np.testing.assert_array_equal(ks, ks_ref)


@pytest.mark.parametrize("name", ["g1_predict_2d", "g1_grid", "g2_predict_512", "g3_predict_6d3o"])
def test_predict_chain(golden, name):
    d = golden(name)
    out = _chain(d)
    for key in ("mu", "var", "std_mu", "std_var", "ucb", "acq"):
        np.testing.assert_array_equal(out[key], d[key], err_msg=key)
    for q in (3, 16):
        sel = O.select_next_batch(d["cand"], out["acq"], d["x"], q)
        np.testing.assert_array_equal(sel, d[f"select_q{q}"])


def test_illcond_chain_runs(golden):
    d = golden("g7_illcond")
    out = _chain(d)
    assert d["cond"].max() > 1e9
    for key in ("mu", "var", "acq"):
        np.testing.assert_array_equal(out[key], d[key], err_msg=key)


def test_mll(golden):
    d = golden("g4_mll")
    for n in (64, 256):
        x, y, pm = d[f"x_{n}"], d[f"y_{n}"], d[f"pm_{n}"]
        for p, ref in zip(d[f"params_{n}"], d[f"mll_{n}"]):
            km = np.zeros((2, n, n))
            try:
                v = O.compute_mll(x, y, km, pm, p[2:4], p[0:2], n)
            except np.linalg.LinAlgError:
                v = np.nan
            if np.isnan(ref):
                assert np.isnan(v)
            else:
                assert v == pytest.approx(ref, rel=1e-12, abs=1e-9)


def test_pareto(golden):
    d = golden("g5_pareto")
    for key in d.files:
        if key.startswith("y_"):
            suffix = key[2:]
            np.testing.assert_array_equal(O.is_pareto_efficient(d[key]), d["mask_" + suffix], err_msg=key)


def test_select_indices_matches_reference_walk(golden):
    d = golden("g1_predict_2d")
    cand, x, acq = d["cand"], d["x"], d["acq"]
    excl = np.array([np.any(np.all(c == x, axis=1)) for c in cand])
    idx = O.select_next_batch_indices(acq, excl, 16)
    np.testing.assert_array_equal(cand[idx], d["select_q16"])


@pytest.mark.parametrize("name", ["g1_predict_2d", "g2_predict_512", "g3_predict_6d3o"])
def test_cpu_ref_matches_oracle(golden, name):
    """oracle/cpu_ref.c (bench.py's timed CPU baseline) against the reference's own outputs."""
    from oracle import cpu_ref
    d = golden(name)
    kinv = kinv_of(d)
    out = cpu_ref.predict_acquire(d["x"], d["y"], d["cand"], kinv, d["pm"], d["pv"], d["ls"],
                                  d["betas"], threads=4, ucb=True)
    from parity import check_predict
    check_predict({k: out[k] for k in ("mu", "var", "ucb", "acq")}, d, d["pv"])
    # the selection itself, with the reference's own acq values as input, is exact
    for q in (3, 16):
        sel = cpu_ref.select(d["acq"], d["cand"], d["x"], q)
        np.testing.assert_array_equal(d["cand"][sel], d[f"select_q{q}"])
