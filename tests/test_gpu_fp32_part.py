"""The fp32 kernel's PART peel (cm32_predict_kernel<DIM, KQV> with KQV < 4, bo_predict_impl.h) at the drop-in
loop's C5 training-set sizes.

C5 (BASELINE.json configs[4]: 6-D / 3 objectives, N_train = 2048, batch q = 16, "fp32 with fp64
reference check") grows N by q = 16 per iteration, so every loop N (2064, 2080, ...) leaves the
fp32 kernel's last 64-row chunk partly padding.  The peel skips the k-quads (16 rows) of that
chunk that hold only padding: their K* rows are exactly 0, so the result must be BIT-IDENTICAL
to the unpeeled kernel (BO_C32_NOPART=1 selects it; the variable is read per launch).

1. bit identity, peeled vs unpeeled, at N = 2049 / 2064 / 2080 / 2090 (1, 1, 2 and 3 live
   k-quads in the last chunk) on a 2^16-candidate slice of the C5 Sobol set: mu, var, acq and the
   top-16 (N = 2100 / 2111, with 52 / 63 rows in the last chunk, have no all-padding k-quad and
   run the unpeeled kernel);
2. the peeled fp32 path against the f64 CPU reference (oracle/cpu_ref.c: update_k_star ->
   update_mean -> update_variance -> standardize -> UCB -> sum, numba_kernels.py:406-570,
   acquisition.py:33-108) on EVERY candidate of C5's 8-GPU shard 0 (2^19) at N = 2064, with the
   per-candidate fp32 bound of tests/test_gpu_c5_shards.py, and the shard's top-16 judged on the
   CPU acquisition array (acquisition.py:116-144)."""
import os
import sys

import numpy as np
import pytest

from parity import check_topq
from fullref import cpu_full

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pytestmark = pytest.mark.gpu

EPS_MU = 1e-5           # as tests/test_gpu_c5_shards.py (|d std_mu|, |d std_var| of the f32 path)
EPS_VAR = 1e-5


@pytest.fixture(scope="module")
def c5():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    import bench
    bo._lib.load()
    cfg = bench.CONFIGS["C5"]
    x0, _, _, _, ls, betas, _, cand = bench.make_config_problem(cfg, 1)
    cs = cand[1]
    # the loop's next points: 96 further members of the candidate set (as scripts/c5_npad_probe.py)
    extra = cs.points(np.random.default_rng(7).choice(cfg["m"], size=96, replace=False))
    return bo, bench, x0, extra, ls, betas, cs


def _problem(c5, n):
    bo, bench, x0, extra, ls, betas, cs = c5
    x = np.concatenate([x0, extra])[:n]
    assert np.unique(x, axis=0).shape[0] == n
    y = bench.toy_function_3d(x)
    pm, pv = y.mean(0), y.var(0)
    return x, y, pm, pv, ls, betas, bench._kinv(x, pv, ls)


def _run(c5, prob, off, cnt, nopart):
    import torch
    bo, cs = c5[0], c5[6]
    x, y, pm, pv, ls, betas, kinv = prob
    if nopart:
        os.environ["BO_C32_NOPART"] = "1"
    try:
        r = bo.predict_acquire(x, y, kinv, cs, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=16,
                               offset=off, count=cnt, mode="fp32")
        torch.cuda.synchronize()
    finally:
        os.environ.pop("BO_C32_NOPART", None)
    return {k: v.cpu().numpy() for k, v in r.items() if not k.startswith("_")}


@pytest.mark.parametrize("n", [2049, 2064, 2080, 2090])
def test_part_bit_identical_to_unpeeled(c5, n):
    prob = _problem(c5, n)
    off, cnt = 3 << 18, 1 << 16
    a = _run(c5, prob, off, cnt, nopart=False)
    b = _run(c5, prob, off, cnt, nopart=True)
    for k in ("mu", "var", "acq", "top_idx", "top_val"):
        assert k in a, k
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), (n, k)


def test_part_c5_shard0_n2064_vs_f64_reference(c5):
    from bayesopt_smart_amd.distributed import shard_range
    cs = c5[6]
    x, y, pm, pv, ls, betas, kinv = prob = _problem(c5, 2064)
    off, cnt = shard_range(cs.n, 0, 8)
    pts = cs.points(np.arange(off, off + cnt))
    ref = cpu_full(("C5shard0_n2064",), x, y, pts, kinv, pm, pv, ls, betas)
    xs = {tuple(p) for p in x}
    excl = np.array([tuple(p) in xs for p in pts])
    got = _run(c5, prob, off, cnt, nopart=False)
    pvc, bc = pv[:, None], betas[:, None]
    dmu = np.abs(got["mu"] - ref["mu"]) / np.sqrt(pvc)
    dvar = np.abs(got["var"] - ref["var"]) / pvc
    print(f"C5 shard 0, N = 2064, fp32 PART: max |d std_mu| {dmu.max():.3e}, "
          f"max |d std_var| {dvar.max():.3e}, max |d acq| {np.abs(got['acq'] - ref['acq']).max():.3e}")
    assert dmu.max() <= EPS_MU, dmu.max()
    assert dvar.max() <= EPS_VAR, dvar.max()
    sv = np.maximum(ref["var"] / pvc, 1e-300)
    tol = np.sum(EPS_MU + bc * np.minimum(np.sqrt(EPS_VAR), EPS_VAR / np.sqrt(sv)), axis=0)
    da = np.abs(got["acq"] - ref["acq"])
    bad = da > tol
    assert not bad.any(), (int(bad.sum()), da[bad][:5], tol[bad][:5])
    check_topq(got["top_idx"] - off, ref["acq"], excl, 16, tol=tol)
