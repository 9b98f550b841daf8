"""Drop-in for bayesopt/bayesian_optimization.py: ``optimize`` and ``BayesianOptimization``
with the reference's signatures, kwargs, ``state`` dict and return values, running the
inner loop (bayesian_optimization.py:108-247) on the MI355X:

  hyper-parameters   Powell on the host, every MLL evaluation one device call (bo_compute_mll)
  update_k/invert_k  device kernels (bo_update_k, bo_invert_k)
  predict+acquire    ONE fused kernel call (bo_predict_acquire) replacing update_k_star ->
                     update_mean -> update_variance -> standardize_objectives -> update_ucb ->
                     update_hypervolume_improvement -> select_next_batch; the N x M k_star
                     buffer of the reference is never allocated
  evaluation         the user's objective on the host (unchanged)

Multi-GPU (one process per GPU, torch.distributed over RCCL): every rank runs the loop; the
candidate set is sharded over the ranks (distributed.shard_range), each rank scores its shard
and ONE all_gather of the per-rank top-q records selects the batch.  The fit is replicated
(rank 0's hyper-parameters are broadcast), the objective is evaluated on rank 0 and its values
broadcast.

Posterior arrays stay in HBM; callbacks receive a ``state`` dict whose array entries are
copied to numpy only when a callback reads them.
"""

from __future__ import annotations

import time
from typing import Any, Callable, List, Optional, Tuple

import numpy as np
import torch

from . import kernels as K
from .acquisition import ExclusionMask, hvi_select_indices, select_indices, update_hypervolume_improvement_exact
from .config import (DEFAULT_BATCH_SIZE, DEFAULT_BETA, DEFAULT_INITIAL_SAMPLES,
                     DEFAULT_LENGTH_SCALE, DEFAULT_PRIOR_MEAN, DEFAULT_PRIOR_VARIANCE,
                     resolve_float_type)
from .device import F64, require_device
from .pareto import compute_pareto_front, print_pareto_analysis
from .predict import CandidateSet, predict_acquire
from . import _lib


class LazyState(dict):
    """``state`` dict (bayesian_optimization.py:226-243); device arrays become numpy on read."""

    def __getitem__(self, key):
        v = dict.__getitem__(self, key)
        if isinstance(v, torch.Tensor):
            v = v.cpu().numpy()
            dict.__setitem__(self, key, v)
        return v

    def get(self, key, default=None):
        return self[key] if key in self else default

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]


class DeviceBuffers:
    """The reference's preallocated posterior arrays (bayesian_optimization.py:355-401), in HBM,
    over `m` candidates (this rank's shard).  k_star (n_obj x T x M) is not among them: the fused
    kernel never materialises it."""

    def __init__(self, n_obj, total, m, dev):
        z = lambda *s: torch.zeros(s, dtype=F64, device=dev)  # noqa: E731
        self.kernel_matrices = z(n_obj, total, total)
        self.mu_objectives = z(n_obj, m)
        self.variance_objectives = z(n_obj, m)
        self.std_mu_objectives = z(n_obj, m)
        self.std_variance_objectives = z(n_obj, m)
        self.ucb = z(n_obj, m)
        self.acquisition_values = z(m)


def _world(group=None):
    """(rank, world size) of the torch.distributed group; (0, 1) when not initialised."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _broadcast_np(arr, group=None, device=None):
    """Broadcast a numpy array (or view) from rank 0 in place; a no-op on one rank.  The
    collective's tensor lives where the backend needs it: on `device` (the backend's HIP device,
    default the current one) for RCCL, on the host for gloo."""
    import torch.distributed as dist
    from .distributed import collectives_on
    if not collectives_on(group) or np.size(arr) == 0:
        return arr
    if dist.get_backend(group) == "nccl":
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    t = torch.as_tensor(np.ascontiguousarray(arr, dtype=np.float64), device=dev)
    dist.broadcast(t, 0, group=group)
    arr[...] = t.cpu().numpy().reshape(np.shape(arr))
    return arr


class DeviceBackend:
    """The device side of one loop iteration (bayesian_optimization.py:115-207) on this rank:

      fit      Powell on the device MLL (every evaluation one bo_compute_mll call), rank 0's
               hyper-parameters broadcast, then update_k + invert_k (bo_update_k, bo_invert_k);
      select   the fused predict + acquisition + top-q (bo_predict_acquire) over this rank's
               candidate shard -- the whole set on one rank; shard_range(M, rank, P) and ONE
               all_gather of the 16-B top-q records with P ranks (sharded_predict_acquire) --
               returning the global batch's candidate indices, identical on every rank.

    `state_arrays` gives the callbacks' mu / variance / acquisition arrays over the whole set:
    this rank's buffers, or the shards gathered (a collective: every rank's loop calls it at the
    same point).

    float_type np.float32 (the reference's float32 branch, config.py:54-66): the fit runs COBYLA
    with the float32 jitters (numba_kernels.py:290-302), invert_k adds 1e-3, and the predict runs
    the f32 matrix-core kernel (mode "fp32") with the variance floor 1e-6."""

    def __init__(self, cands, n_obj, total_samples, device=None, buffers=None, group=None, float_type=None):
        from .distributed import shard_range
        self.dev = require_device(device)
        self.float_type = resolve_float_type(float_type)
        self.mode = "fp32" if self.float_type == np.float32 else "auto"
        self.cands = cands
        self.group = group
        self.rank, self.world = _world(group)
        self.offset, self.count = shard_range(cands.n, self.rank, self.world)
        if buffers is None:
            buffers = DeviceBuffers(n_obj, total_samples, self.count, self.dev)
        self.bufs = buffers
        self._lu_hint = None           # per objective: the previous invert_k took the LU path
        self.inverse_paths = []
        self._excl_mask = None         # the shard's ExclusionMask (exact-HVI selection)

    def fit(self, x_vector, y_vector, n, prior_mean, prior_variance, length_scales):
        """Returns (Powell's OptimizeResult, fitted device state, time after the Powell fit)."""
        xd = torch.as_tensor(np.ascontiguousarray(x_vector[:n], dtype=np.float64), device=self.dev)
        yd = torch.as_tensor(np.ascontiguousarray(y_vector[:n], dtype=np.float64), device=self.dev)
        optimized = K.optimize_hyperparams_mll(xd, yd, self.bufs.kernel_matrices, prior_mean,
                                               prior_variance, length_scales, n, float_type=self.float_type)
        _broadcast_np(length_scales, self.group, self.dev)
        _broadcast_np(prior_variance, self.group, self.dev)
        t1 = time.perf_counter()
        K.update_k(self.bufs.kernel_matrices, xd, 0, n, prior_variance, length_scales)
        # an objective whose Cholesky failed last iteration (Powell-fitted length scales drive
        # cond(K + 1e-6 I) past 1e16) fails again: when all did, go straight to the
        # blocked LU -- gesv's algorithm, the reference's own -- without the doomed attempt
        from .distributed import collectives_on
        if self.world > 1 and collectives_on(self.group):
            kinv = self._invert_split(n)
        else:
            paths = []
            kinv = K.invert_k(n, self.bufs.kernel_matrices, float_type=self.float_type, lu_hint=self._lu_hint,
                              paths=paths)
            self._lu_hint = [p != 0 for p in paths]
            self.inverse_paths = paths
        torch.cuda.synchronize(self.dev)
        return optimized, (xd, yd, kinv), t1

    def _invert_split(self, n):
        """invert_k with the objectives split over the ranks (objective o on rank o mod P), each
        K^-1 then broadcast from its rank (one broadcast per objective: n^2 doubles, 2 MiB at C3).
        Each objective's inverse is the same per-objective device computation as in the batched
        single-rank call, so every rank holds the single-rank K^-1 bit for bit."""
        import torch.distributed as dist
        km = self.bufs.kernel_matrices
        n_obj = km.shape[0]
        mine = [o for o in range(n_obj) if o % self.world == self.rank]
        kinv = torch.empty((n_obj, n, n), dtype=F64, device=self.dev)
        hint = self._lu_hint or [False] * n_obj
        paths = [0] * n_obj
        if mine:
            sub = km[mine] if len(mine) > 1 else km[mine[0]:mine[0] + 1]
            p = []
            got = K.invert_k(n, sub.contiguous(), float_type=self.float_type, lu_hint=[hint[o] for o in mine],
                             paths=p)
            for i, o in enumerate(mine):
                kinv[o] = got[i]
                paths[o] = p[i]
        nccl = dist.get_backend(self.group) == "nccl"
        for o in range(n_obj):
            src = o % self.world                    # a group rank; broadcast takes the global one
            if self.group is not None:
                src = dist.get_global_rank(self.group, src)
            if nccl:
                dist.broadcast(kinv[o], src=src, group=self.group)
            else:                                   # gloo: the collective on a host copy
                h = kinv[o].cpu()
                dist.broadcast(h, src=src, group=self.group)
                kinv[o].copy_(h)
        # the path hints follow the objectives this rank inverts (o mod P is fixed)
        self._lu_hint = [paths[o] != 0 if o in mine else hint[o] for o in range(n_obj)]
        self.inverse_paths = paths
        return kinv

    def _outputs(self):
        b = self.bufs
        return {"mu": b.mu_objectives, "var": b.variance_objectives, "std_mu": b.std_mu_objectives,
                "std_var": b.std_variance_objectives, "ucb": b.ucb, "acq": b.acquisition_values}

    def select(self, fitted, prior_mean, prior_variance, length_scales, betas, batch_size, evaluated,
               acquisition="sum_ucb", y_evaluated=None, reference_point=None):
        """Global candidate indices of the next batch (select_next_batch's order, the evaluated
        points excluded).  "sum_ucb" is the reference's acquisition (acquisition.py:89-108, fused
        top-q); "hvi" replaces the acquisition array with the exact hypervolume improvement of the
        UCB vectors over the Pareto front of `y_evaluated` above `reference_point`."""
        if acquisition not in ("sum_ucb", "hvi"):
            raise ValueError(f"unknown acquisition {acquisition!r} (expected 'sum_ucb' or 'hvi')")
        xd, yd, kinv = fitted
        out = self._outputs()
        if acquisition == "sum_ucb" and batch_size <= _lib.MAX_TOPQ:
            from .distributed import sharded_predict_acquire
            _, (_, idx) = sharded_predict_acquire(xd, yd, kinv, self.cands, prior_mean, prior_variance,
                                                  length_scales, betas, batch_size, outputs=tuple(out),
                                                  group=self.group, device=self.dev, out=out, mode=self.mode,
                                                  float_type=self.float_type)
            return np.asarray(idx, dtype=np.int64)
        predict_acquire(xd, yd, kinv, self.cands, prior_mean, prior_variance, length_scales, betas,
                        outputs=tuple(out), topq=0, offset=self.offset, count=self.count, out=out,
                        device=self.dev, mode=self.mode, float_type=self.float_type)
        if acquisition == "hvi" and batch_size <= _lib.MAX_TOPQ:
            # the exact HVI and its top-q with exclusion in one device pass over this shard, then
            # the fused path's exchange
            # the shard's exclusion mask persists across iterations: only the new batch's rows
            # are added to it (ExclusionMask)
            if self._excl_mask is None:
                self._excl_mask = ExclusionMask(self.cands, self.offset, self.count, self.dev)
            rec = hvi_select_indices(self.bufs.acquisition_values, self.bufs.ucb, y_evaluated,
                                     len(y_evaluated), reference_point, prior_mean, prior_variance,
                                     self.cands, evaluated, batch_size, offset=self.offset,
                                     return_record=True, mask=self._excl_mask)
            from .distributed import collectives_on, exchange_topq_rec
            if not collectives_on(self.group):
                idx = rec[batch_size:].view(torch.int64).cpu().numpy()
                return idx[idx >= 0]
            return np.asarray(exchange_topq_rec(rec, batch_size, self.group)[1], dtype=np.int64)
        if acquisition == "hvi":
            update_hypervolume_improvement_exact(self.bufs.acquisition_values, self.bufs.ucb, y_evaluated,
                                                 len(y_evaluated), reference_point, prior_mean,
                                                 prior_variance)
        # batches above BO_MAX_TOPQ: rounds of the standalone device selection (over the gathered
        # array when sharded)
        from .distributed import collectives_on
        acq = self.bufs.acquisition_values if not collectives_on(self.group) else \
            torch.as_tensor(self.state_arrays()["acquisition_values"], device=self.dev)
        return select_indices(acq, self.cands, evaluated, batch_size)

    def state_arrays(self):
        b = self.bufs
        arrs = {"mu_objectives": b.mu_objectives, "variance_objectives": b.variance_objectives,
                "acquisition_values": b.acquisition_values}
        from .distributed import collectives_on, gather_shards
        if not collectives_on(self.group):
            return arrs
        return {k: gather_shards(v, self.cands.n, self.group) for k, v in arrs.items()}


def optimize(x_vector, y_vector, kernel_matrices, k_star, mu_objectives, variance_objectives,
             std_mu_objectives, std_variance_objectives, ucb, acquisition_values, input_space,
             prior_mean, prior_variance, reference_point, n_evaluations, total_samples,
             n_objectives, function, betas, length_scales, batch_size, bounds,
             callbacks: Optional[List[Callable]] = None, *,
             acquisition: str = "sum_ucb", group=None, backend=None,
             float_type=None) -> Tuple[np.ndarray, np.ndarray, int]:
    """bayesian_optimization.py:51-247 with the reference's argument list.

    `kernel_matrices` and the posterior arrays may be HIP tensors (in place) or numpy arrays;
    `k_star` is accepted for signature compatibility and not used (nothing N x M is
    materialised); `input_space` may be a CandidateSet, a device tensor or the reference's
    int64 numpy array.  Returns (x_vector, y_vector, last_eval + 1) like the reference
    (including its count quirk, :247).

    With torch.distributed initialised (one process per GPU) every rank runs this loop over its
    shard of the candidates (module docstring); the posterior arrays given here are then not
    filled (each rank holds its shard), the state dict's arrays are the gathered whole.  `group`
    selects the process group; `backend` replaces the device side (DeviceBackend's interface:
    fit / select / state_arrays / cands / rank / world / bufs).  `float_type` np.float32 runs the
    reference's float32 branch (DeviceBackend).

    Callbacks with several ranks: the state arrays are the shards gathered, a collective; whether
    to gather is decided once, collectively (any rank with callbacks), so that a callback
    registered on rank 0 only keeps every rank's collectives matched.
    """
    del k_star, n_objectives, bounds  # unused, as in the reference (reference_point too, unless
    #                                   acquisition="hvi", the exact hypervolume improvement)
    n_obj = len(prior_mean)
    if backend is None:
        dev = require_device()
        cands = input_space if isinstance(input_space, CandidateSet) else CandidateSet.explicit(input_space, dev)
        from .distributed import shard_range
        _, world = _world(group)
        cnt = shard_range(cands.n, _world(group)[0], world)[1]

        def dev_buf(a, shape):
            if isinstance(a, torch.Tensor) and a.device.type == "cuda" and tuple(a.shape) == shape:
                return a
            return torch.zeros(shape, dtype=F64, device=dev)

        bufs = DeviceBuffers.__new__(DeviceBuffers)
        bufs.kernel_matrices = dev_buf(kernel_matrices, (n_obj, total_samples, total_samples))
        bufs.mu_objectives = dev_buf(mu_objectives, (n_obj, cnt))
        bufs.variance_objectives = dev_buf(variance_objectives, (n_obj, cnt))
        bufs.std_mu_objectives = dev_buf(std_mu_objectives, (n_obj, cnt))
        bufs.std_variance_objectives = dev_buf(std_variance_objectives, (n_obj, cnt))
        bufs.ucb = dev_buf(ucb, (n_obj, cnt))
        bufs.acquisition_values = dev_buf(acquisition_values, (cnt,))
        backend = DeviceBackend(cands, n_obj, total_samples, dev, bufs, group, float_type=float_type)
    cands, rank, world = backend.cands, backend.rank, backend.world
    gather = bool(callbacks)
    bgroup = getattr(backend, "group", group)
    from .distributed import collectives_on
    coll = collectives_on(bgroup)
    if coll:                            # any rank with callbacks: every rank joins the gathers
        import torch.distributed as dist
        if dist.get_backend(bgroup) == "nccl":      # RCCL: the flag on the backend's HIP device
            bdev = getattr(backend, "dev", None)
            fdev = torch.device(bdev) if bdev is not None else torch.device("cuda", torch.cuda.current_device())
        else:
            fdev = torch.device("cpu")
        flag = torch.tensor([1.0 if callbacks else 0.0], dtype=torch.float64, device=fdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=bgroup)
        gather = bool(flag.item())

    last_eval = 0
    for current_eval in range(n_evaluations, total_samples, batch_size):
        iter_start = time.perf_counter()
        t0 = time.perf_counter()
        optimized, fitted, t1 = backend.fit(x_vector, y_vector, current_eval, prior_mean, prior_variance,
                                            length_scales)
        t2 = time.perf_counter()
        idx = backend.select(fitted, prior_mean, prior_variance, length_scales, betas, batch_size,
                             x_vector[:current_eval], acquisition, y_vector[:current_eval], reference_point)
        x_next = cands.points(idx) if idx.size else np.zeros((0, cands.dim), dtype=np.int64)
        t3 = time.perf_counter()
        for b_idx, point in enumerate(x_next):
            x_vector[current_eval + b_idx] = point
            if rank == 0:       # the user's objective, once per point (bayesian_optimization.py:213-216)
                y_vector[current_eval + b_idx] = function(point)
        if coll:
            _broadcast_np(y_vector[current_eval:current_eval + len(x_next)], bgroup,
                          getattr(backend, "dev", None))
        last_eval = current_eval
        t4 = time.perf_counter()
        if gather:
            arrs = backend.state_arrays()
        if callbacks:
            state = LazyState({
                "iteration": current_eval,
                "n_evaluations": current_eval + batch_size,
                "x_vector": x_vector[: current_eval + batch_size],
                "y_vector": y_vector[: current_eval + batch_size],
                "mu_objectives": arrs["mu_objectives"],
                "variance_objectives": arrs["variance_objectives"],
                "acquisition_values": arrs["acquisition_values"],
                "x_next": x_next,
                "hyperparams": optimized.x,
                # the reference's keys; update_k_star (its "kernels", :145-153) is fused into the
                # predict call and so counted under "acquisition" here
                "timings": {"hyperparams": t1 - t0, "kernels": t2 - t1, "acquisition": t3 - t2,
                            "eval": t4 - t3, "total": t4 - iter_start},
            })
            for cb in callbacks:
                cb(state)
    bufs = getattr(backend, "bufs", None)
    if bufs is not None and world == 1:
        if isinstance(kernel_matrices, np.ndarray):   # the reference mutates it in place (update_k)
            kernel_matrices[...] = bufs.kernel_matrices.cpu().numpy().reshape(kernel_matrices.shape)
        for name, a in (("mu", mu_objectives), ("var", variance_objectives), ("smu", std_mu_objectives),
                        ("svar", std_variance_objectives), ("ucb", ucb), ("acq", acquisition_values)):
            if isinstance(a, np.ndarray):   # numpy callers get their arrays filled, as in the reference
                src = {"mu": bufs.mu_objectives, "var": bufs.variance_objectives,
                       "smu": bufs.std_mu_objectives, "svar": bufs.std_variance_objectives,
                       "ucb": bufs.ucb, "acq": bufs.acquisition_values}[name]
                a[...] = src.cpu().numpy()
    return x_vector, y_vector, last_eval + 1


def _check_limits(n_obj, dim, total_samples, batch_size, acquisition="sum_ucb"):
    """Fail in the constructor -- before any objective evaluation -- on shapes the device path
    cannot run (the reference would hit them only mid-loop, if at all)."""
    if not 1 <= n_obj <= _lib.MAX_OBJ:
        raise ValueError(f"n_objectives must be in [1, {_lib.MAX_OBJ}] (got {n_obj})")
    if acquisition == "hvi" and n_obj > 4:
        raise ValueError(f"acquisition='hvi' supports at most 4 objectives (got {n_obj}): the exact "
                         "hypervolume improvement's box decomposition is limited to n_obj <= 4")
    if not 1 <= dim <= _lib.MAX_DIM:
        raise ValueError(f"the input dimension must be in [1, {_lib.MAX_DIM}] (got {dim})")
    if batch_size < 1:
        raise ValueError("batch_size must be >= 1")
    d = _lib.PredictDesc()
    d.n_obj, d.dim, d.n_train, d.n_cand, d.cand_kind, d.topq = n_obj, dim, total_samples, 1, _lib.CAND_GRID, 0
    for k in range(dim):
        d.grid_shape[k] = 1
    lib = _lib.load()
    if lib.bo_predict_workspace_size(d) == 0 or lib.bo_invert_k_workspace_size(n_obj, total_samples) == 0:
        raise ValueError(f"total_samples = {total_samples} exceeds the device path's limits "
                         f"(predict: N <= 16384 and n_obj N^2 doubles < 2 GiB)")


class BayesianOptimization:
    """bayesian_optimization.py:250-488 — same constructor, kwargs and methods.

    Extra kwargs (not in the reference): ``input_space`` (explicit [M, d] candidates, e.g.
    a Sobol set, or a CandidateSet such as CandidateSet.sobol_set(...), instead of the integer
    grid), ``device``, ``acquisition`` ("sum_ucb", the reference's default, or "hvi": exact
    hypervolume improvement of the UCB vectors over the evaluated Pareto front),
    ``reference_point`` (the HVI reference point; the reference fixes it at zeros and never uses
    it, bayesian_optimization.py:425), ``group`` (the torch.distributed process group of a
    multi-GPU run; default: the world when initialised), ``float_type`` (np.float64, the default
    of config.NUMBA_FLOAT_TYPE, or np.float32: the reference's float32 branch -- config.py:54-66
    jitters and variance floor, COBYLA for the fit, float32 host arrays -- with the predict on the
    f32 matrix cores) and ``initial_points`` ([n0, d] points evaluated as the initial design
    instead of the Latin hypercube).
    With several ranks, each holds its shard of the posterior arrays, the initial design is drawn
    and evaluated on rank 0 (every rank draws the same RNG numbers, so the RNG stays in step) and
    broadcast, and the loop runs as `optimize` describes.
    """

    def __init__(self, function: Callable[[np.ndarray], np.ndarray], bounds: List[Tuple[int, int]],
                 n_objectives: int = 3, n_iterations: int = 10, **kwargs: Any):
        self.device = require_device(kwargs.get("device"))
        self.group = kwargs.get("group")
        self.float_type = resolve_float_type(kwargs.get("float_type"))
        ft = self.float_type
        self.function = function
        self.bounds = bounds
        self.n_objectives = n_objectives
        self.n_iterations = n_iterations
        cb = kwargs.get("callbacks", None)
        self.callbacks = [] if cb is None else (cb if isinstance(cb, list) else [cb])
        self.prior_mean = np.array(kwargs.get("prior_mean", [DEFAULT_PRIOR_MEAN] * n_objectives), dtype=ft)
        self.prior_variance = np.array(kwargs.get("prior_variance", [DEFAULT_PRIOR_VARIANCE] * n_objectives),
                                       dtype=ft)
        self.length_scales = np.array(kwargs.get("length_scales", [DEFAULT_LENGTH_SCALE] * n_objectives), dtype=ft)
        self.betas = np.array(kwargs.get("betas", [DEFAULT_BETA] * n_objectives), dtype=ft)
        self.batch_size = kwargs.get("batch_size", DEFAULT_BATCH_SIZE)
        init_pts = kwargs.get("initial_points")
        if init_pts is not None:
            init_pts = np.asarray(init_pts)
            if init_pts.ndim != 2 or init_pts.shape[1] != len(bounds):
                raise ValueError("initial_points must be [n0, len(bounds)]")
        self.initial_samples = init_pts.shape[0] if init_pts is not None else \
            kwargs.get("initial_samples", DEFAULT_INITIAL_SAMPLES)
        self.dim = len(bounds)
        explicit = kwargs.get("input_space")
        if explicit is None:
            self.candidates = CandidateSet.grid(bounds)
        elif isinstance(explicit, CandidateSet):
            self.candidates = explicit
        else:
            self.candidates = CandidateSet.explicit(explicit, self.device)
        self._input_space = None
        self.total_samples = self.initial_samples + self.n_iterations * self.batch_size
        self.acquisition = kwargs.get("acquisition", "sum_ucb")
        if self.acquisition not in ("sum_ucb", "hvi"):
            raise ValueError(f"unknown acquisition {self.acquisition!r} (expected 'sum_ucb' or 'hvi')")
        _check_limits(n_objectives, self.dim, self.total_samples, self.batch_size, self.acquisition)
        self.x_vector = np.zeros((self.total_samples, self.dim), dtype=ft)
        self.y_vector = np.zeros((self.total_samples, n_objectives), dtype=ft)
        self._backend = DeviceBackend(self.candidates, n_objectives, self.total_samples, self.device,
                                      group=self.group, float_type=ft)
        self._buffers = self._backend.bufs
        self.k_star = None   # never materialised (the reference allocates n_obj x T x M here)
        rank, world = _world(self.group)
        # the objective runs on rank 0 only; the other ranks draw the same LHS numbers (their RNG
        # stays in step with rank 0's) and receive rank 0's design and values
        fn = self.function if rank == 0 else (lambda _p: np.zeros(n_objectives))
        if init_pts is not None:
            for i in range(self.initial_samples):
                self.x_vector[i] = init_pts[i]
                self.y_vector[i] = fn(self.x_vector[i])
            self.n_evaluations = self.initial_samples
        else:
            self.n_evaluations = K.initialize_lhs_integer(self.x_vector, self.y_vector,
                                                          np.array(self.bounds, dtype=np.int64),
                                                          fn, self.initial_samples)
        _broadcast_np(self.x_vector[: self.n_evaluations], self.group, self.device)
        _broadcast_np(self.y_vector[: self.n_evaluations], self.group, self.device)
        if np.all(self.prior_mean == DEFAULT_PRIOR_MEAN):
            self.prior_mean = K.compute_prior_mean(self.y_vector, self.n_evaluations, n_objectives).astype(ft)
        if np.all(self.prior_variance == DEFAULT_PRIOR_VARIANCE):
            self.prior_variance = K.compute_prior_variance(self.y_vector, self.n_evaluations,
                                                           n_objectives).astype(ft)
        self.reference_point = np.array(kwargs.get("reference_point", [0.0] * n_objectives), dtype=ft)

    # the reference's preallocated arrays, materialised on the host on demand
    @property
    def input_space(self):
        if self._input_space is None:
            self._input_space = self.candidates.materialize(self.device).cpu().numpy()
        return self._input_space

    def _np(self, name):
        return getattr(self._buffers, name).cpu().numpy()

    kernel_matrices = property(lambda self: self._np("kernel_matrices"))
    mu_objectives = property(lambda self: self._np("mu_objectives"))
    variance_objectives = property(lambda self: self._np("variance_objectives"))
    std_mu_objectives = property(lambda self: self._np("std_mu_objectives"))
    std_variance_objectives = property(lambda self: self._np("std_variance_objectives"))
    ucb = property(lambda self: self._np("ucb"))
    acquisition_values = property(lambda self: self._np("acquisition_values"))

    def optimize(self) -> None:
        """bayesian_optimization.py:427-463."""
        b = self._buffers
        self.x_vector, self.y_vector, self.n_evaluations = optimize(
            x_vector=self.x_vector, y_vector=self.y_vector, kernel_matrices=b.kernel_matrices,
            k_star=None, mu_objectives=b.mu_objectives, variance_objectives=b.variance_objectives,
            std_mu_objectives=b.std_mu_objectives, std_variance_objectives=b.std_variance_objectives,
            ucb=b.ucb, acquisition_values=b.acquisition_values, input_space=self.candidates,
            prior_mean=self.prior_mean, prior_variance=self.prior_variance,
            reference_point=self.reference_point, n_evaluations=self.n_evaluations,
            total_samples=self.total_samples, n_objectives=self.n_objectives, function=self.function,
            betas=self.betas, length_scales=self.length_scales, batch_size=self.batch_size,
            bounds=self.bounds, callbacks=self.callbacks if self.callbacks else None,
            acquisition=self.acquisition, group=self.group, backend=self._backend,
            float_type=self.float_type)

    def pareto_analysis(self) -> np.ndarray:
        """bayesian_optimization.py:465-488."""
        ey = self.y_vector[: self.n_evaluations]
        ex = self.x_vector[: self.n_evaluations]
        px, py = compute_pareto_front(ex, ey)
        print_pareto_analysis(px, py)
        return py
