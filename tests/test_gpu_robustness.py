"""GPU parity outside the benchmark shapes: coordinates far from the origin (the centred
exponent), the dot-form gate's fallback for extents far above the length scale, and training
sets too large for the kernel's LDS (rows and alpha streamed from global memory; the reference's
update_k_star / update_mean / update_variance, numba_kernels.py:406-535, have no N cap).

Every case is checked on every candidate against oracle/cpu_ref.c (tests/fullref.py) with the
SURVEY.md §8c tolerances (tests/parity.py), and the top-q against the CPU acquisition array."""

import numpy as np
import pytest

from oracle import oracle_np as O
from parity import check_predict, check_topq
from fullref import cpu_full

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


def _kinv(x, pv, ls):
    n, n_obj = x.shape[0], len(pv)
    km = np.zeros((n_obj, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    cond = max(np.linalg.cond(km[o] + 1e-6 * np.eye(n)) for o in range(n_obj)) if n <= 1500 else None
    return O.invert_k(n, km), cond


def _check(bo, key, x, y, cand, cands, ls, betas, q, mode="auto", count=None):
    import torch
    pm, pv = y.mean(0), y.var(0)
    kinv, cond = _kinv(x, pv, ls)
    if cond is not None:
        assert cond < 1e7, cond
    r = bo.predict_acquire(x, y, kinv, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=q,
                           mode=mode, count=count)
    torch.cuda.synchronize()
    got = {k: r[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx")}
    ref = cpu_full(key, x, y, cand, kinv, pm, pv, ls, betas)
    check_predict({k: got[k] for k in ("mu", "var", "acq")}, ref, pv)
    xs = {tuple(p) for p in np.asarray(x, dtype=np.float64)}
    excl = np.array([tuple(c) in xs for c in np.asarray(cand, dtype=np.float64)])
    check_topq(got["top_idx"], ref["acq"], excl, q)
    return got


@pytest.mark.parametrize("kind", ["f64", "i64"])
@pytest.mark.parametrize("ls", [1.0, 5.0])
@pytest.mark.parametrize("mode", ["auto", "dense"])
def test_coordinates_offset_1e6(bo, kind, ls, mode):
    """Explicit candidates on a 40 x 40 integer lattice shifted by 10^6 (|x|^2 ~ 1e12): the
    uncentred dot-form exponent would lose ~1e-4 absolute; centred on a training point it is
    exact to ~1e-12."""
    rng = np.random.default_rng(int(ls * 10) + (kind == "i64"))
    off = 1_000_000
    grid = O.grid_points([(off, off + 40), (off + 7, off + 47)])
    cand = grid if kind == "i64" else grid.astype(np.float64)
    x = grid[rng.choice(grid.shape[0], 40 if ls == 5.0 else 150, replace=False)].astype(np.float64)
    y = np.stack([-((x[:, 0] - off - 20) ** 2) + 100, -((x[:, 1] - off - 30) ** 2) + 20], axis=1)
    cands = bo.CandidateSet.explicit(cand)
    _check(bo, ("off", kind, ls), x, y, cand, cands, np.array([ls, ls]), np.array([2.0, 1.0]), 8, mode)


def test_wide_extent_uses_direct_exponent(bo):
    """Training points spread over [0, 2e5]^3 with length scale 1: max|nl2| (|x - z|^2 + |c - z|^2)
    exceeds the dot-form gate, so the kernel takes the direct |x - c|^2 exponent; the candidates
    sit within a few units of the training points, where K* is far from 0."""
    rng = np.random.default_rng(3)
    x = rng.integers(0, 200_000, size=(64, 3)).astype(np.float64)
    nb = np.stack(np.meshgrid(*[np.arange(-3, 4)] * 3, indexing="ij"), -1).reshape(-1, 3)
    cand = np.unique((x[:, None, :] + nb[None, :, :]).reshape(-1, 3), axis=0)
    y = rng.normal(size=(64, 2)) * 30
    cands = bo.CandidateSet.explicit(cand)
    _check(bo, "wide", x, y, cand, cands, np.array([1.0, 1.5]), np.array([2.0, 2.0]), 5)


@pytest.mark.parametrize("mode", ["auto", "dense"])
def test_large_n_6d_3obj_global_rows(bo, mode):
    """N = 3000, 6-D / 3 objectives: rows + alpha exceed the 160 KiB LDS, the kernel streams them
    from global memory (no N cap); Sobol candidates in [0, 300)^6, length scale 40."""
    from scipy.stats import qmc
    rng = np.random.default_rng(30)
    cand = qmc.Sobol(6, scramble=False).random(1 << 14) * 300.0
    x = qmc.Sobol(6, scramble=True, seed=5).random(3000) * 300.0
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20,
                  -((x[:, 2] - 5) ** 2) + 120], axis=1)
    x[:40] = cand[rng.choice(cand.shape[0], 40, replace=False)]          # some evaluated candidates
    y[:40] = np.stack([-((x[:40, 0] - 150) ** 2) + 100, -((x[:40, 1] - 150) ** 2) + 20,
                       -((x[:40, 2] - 5) ** 2) + 120], axis=1)
    cands = bo.CandidateSet.explicit(cand)
    _check(bo, ("n3000",), x, y, cand, cands, np.full(3, 40.0), np.full(3, 2.0), 16, mode)


def test_large_n_2d_grid_global_rows(bo):
    """N = 6000 on the reference's integer 'ij' grid (1024 x 1024), 2 objectives: beyond the LDS
    budget of the separable grid path, so the global-rows kernel scores the grid; 32768
    candidates of it (rows 0-31) against the CPU reference."""
    rng = np.random.default_rng(60)
    side = 1024
    lin = rng.choice(side * side, size=6000, replace=False)
    lin[:30] = rng.choice(32 * side, 30, replace=False)                    # evaluated candidates
    lin = np.unique(lin)
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20], axis=1)
    cands = bo.CandidateSet.grid([(0, side), (0, side)])
    m = 32 * side
    cand = np.stack([np.arange(m) // side, np.arange(m) % side], axis=1)
    _check(bo, ("n6000",), x, y, cand, cands, np.array([3.0, 3.0]), np.array([2.0, 2.0]), 3,
           count=m)


def test_workspace_plan_has_no_n_cap(bo):
    """bo_predict_workspace_size accepts N far beyond the LDS budget (global-rows plan)."""
    lib = bo._lib.load()
    from bayesopt_smart_amd.predict import _fill_desc
    import torch
    for n, dim, n_obj in ((4000, 6, 3), (8000, 2, 2)):
        x = torch.zeros((n, dim), dtype=torch.float64, device="cuda")
        y = torch.zeros((n, n_obj), dtype=torch.float64, device="cuda")
        k = torch.zeros((n_obj, 1, 1), dtype=torch.float64, device="cuda")
        c = bo.CandidateSet.grid([(0, 64)] * dim)
        d = _fill_desc(x, y, k, c, [0.0] * n_obj, [1.0] * n_obj, [1.0] * n_obj, [1.0] * n_obj, 0, 1024,
                       None, 3)
        assert lib.bo_predict_workspace_size(d) > 0
