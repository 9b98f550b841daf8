"""Fused GP predict + acquisition over a candidate set (the north-star hot path).

``predict_acquire`` is the host side of ``bo_predict_acquire`` (include/bo_amd.h): one
call scores a shard of candidates -- posterior mean and variance
(bayesopt/numba_kernels.py:450-535), standardisation (:538-570), per-objective UCB and
the reference's summed-UCB "hypervolume improvement" (bayesopt/acquisition.py:33-108) --
and returns the shard's top-q selection with evaluated points excluded
(bayesopt/acquisition.py:116-144).  No N x M k_star array exists anywhere.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from .device import F64, Workspace, as_dev, ptr, require_device, stream_handle

OUTPUT_NAMES = ("mu", "var", "std_mu", "std_var", "ucb", "acq")


@dataclass
class CandidateSet:
    """Candidates scored by the hot path.

    kind ``grid``: the reference's integer 'ij' meshgrid (bayesian_optimization.py:338-340),
    generated on the device from the linear index (no candidate array in HBM);
    kind ``sobol``: the unscrambled Sobol sequence of scipy.stats.qmc.Sobol(d, scramble=False)
    mapped to lo + u * scale, generated on the device from the index (bit-identical to scipy;
    each candidate shard generates its own index range);
    kind ``i64``/``f64``: an explicit [M, d] device array (the reference's input_space).
    """

    kind: str
    n: int
    dim: int
    tensor: Optional[torch.Tensor] = None
    lo: Optional[Sequence[int]] = None
    shape: Optional[Sequence[int]] = None
    sobol: Optional[object] = None          # _lib.SobolDesc (kind "sobol")

    @staticmethod
    def grid(bounds):
        lo = [int(b[0]) for b in bounds]
        shape = [int(b[1]) - int(b[0]) for b in bounds]
        n = int(np.prod(shape, dtype=np.int64))
        return CandidateSet("grid", n, len(bounds), lo=lo, shape=shape)

    @staticmethod
    def sobol_set(dim, n, lo=0.0, scale=1.0, bits=30):
        """Points 0 .. n-1 of scipy.stats.qmc.Sobol(dim, scramble=False, bits=bits).random(n),
        as lo + u * scale per dimension (scalars or sequences)."""
        if not 1 <= dim <= _lib.MAX_DIM or not 1 <= bits <= 32 or n > (1 << bits):
            raise ValueError("Sobol set needs 1 <= dim <= 8, 1 <= bits <= 32 and n <= 2^bits")
        d = _lib.SobolDesc()
        d.bits = bits
        lo = np.broadcast_to(np.asarray(lo, dtype=np.float64), (dim,))
        scale = np.broadcast_to(np.asarray(scale, dtype=np.float64), (dim,))
        for k in range(dim):
            d.lo[k] = float(lo[k])
            d.scale[k] = float(scale[k])
        return CandidateSet("sobol", int(n), int(dim), sobol=d)

    @staticmethod
    def explicit(points, device=None):
        dev = require_device(device)
        if isinstance(points, torch.Tensor):
            is_int = not points.is_floating_point()
        else:
            points = np.asarray(points)
            is_int = np.issubdtype(points.dtype, np.integer)
        dtype = torch.int64 if is_int else F64
        t = as_dev(points, dev, dtype)
        if t.dim() != 2:
            raise ValueError("candidates must be [M, d]")
        return CandidateSet("i64" if is_int else "f64", t.shape[0], t.shape[1], tensor=t)

    @property
    def kind_code(self):
        return {"i64": _lib.CAND_I64, "f64": _lib.CAND_F64, "grid": _lib.CAND_GRID,
                "sobol": _lib.CAND_SOBOL}[self.kind]

    @property
    def cand_arg(self):
        """The `cand` argument of the ABI calls: device array pointer, or the host Sobol desc."""
        import ctypes
        if self.kind == "sobol":
            return ctypes.cast(ctypes.pointer(self.sobol), ctypes.c_void_p).value
        return None if self.tensor is None else self.tensor.data_ptr()

    def points(self, idx):
        """Coordinates of global candidate indices (numpy [k, d]; int64 for grid/i64)."""
        idx = np.ascontiguousarray(idx, dtype=np.int64).ravel()
        if self.kind == "sobol":
            import ctypes
            out = np.empty((idx.size, self.dim), dtype=np.float64)
            _lib.check(_lib.load().bo_sobol_points(
                ctypes.byref(self.sobol), self.dim, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                idx.size, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))), "bo_sobol_points")
            return out
        if self.kind == "grid":
            out = np.empty((idx.size, self.dim), dtype=np.int64)
            rem = idx.copy()
            for k in range(self.dim - 1, -1, -1):
                out[:, k] = self.lo[k] + rem % self.shape[k]
                rem //= self.shape[k]
            return out
        return self.tensor[torch.as_tensor(idx, device=self.tensor.device)].cpu().numpy()

    def materialize(self, device=None):
        """Explicit [M, d] tensor: int64 for a grid (the reference's input_space), f64 Sobol."""
        if self.kind == "sobol":
            return torch.as_tensor(self.points(np.arange(self.n)), device=require_device(device))
        if self.kind != "grid":
            return self.tensor
        dev = require_device(device)
        ranges = [torch.arange(l, l + s, device=dev, dtype=torch.int64) for l, s in zip(self.lo, self.shape)]
        mesh = torch.meshgrid(*ranges, indexing="ij")
        return torch.stack([m.reshape(-1) for m in mesh], dim=-1).contiguous()


def _fill_desc(x_train, y_train, kinv, cands, pm, pv, ls, betas, offset, count, excl, topq):
    d = _lib.PredictDesc()
    n_obj = len(pm)
    if not 1 <= n_obj <= _lib.MAX_OBJ:
        raise ValueError(f"n_objectives must be in [1, {_lib.MAX_OBJ}]")
    if not 1 <= cands.dim <= _lib.MAX_DIM:
        raise ValueError(f"dimension must be in [1, {_lib.MAX_DIM}]")
    n = x_train.shape[0]
    d.n_obj = n_obj
    d.dim = cands.dim
    d.n_train = n
    d.x_train = ptr(x_train)
    d.y_train = ptr(y_train)
    d.ld_y = y_train.stride(0)
    d.kinv = ptr(kinv)
    d.ld_k = kinv.shape[-1]
    d.cand_kind = cands.kind_code
    d.n_cand = count
    d.cand_offset = offset
    if cands.kind == "grid":
        for k in range(cands.dim):
            d.grid_lo[k] = cands.lo[k]
            d.grid_shape[k] = cands.shape[k]
        d.cand = None
    elif cands.kind == "sobol":
        d.cand = cands.cand_arg                  # host bo_sobol_desc, read during the call
    else:
        # explicit candidates: the call sees rows [offset, offset + count)
        d.cand = cands.tensor.data_ptr() + offset * cands.dim * cands.tensor.element_size()
        d.cand_offset = offset
    if excl is not None:
        d.excl_points = ptr(excl)
        d.n_excl = excl.shape[0]
    for o in range(n_obj):
        d.prior_mean[o] = float(pm[o])
        d.prior_var[o] = float(pv[o])
        d.length_scale[o] = float(ls[o])
        d.beta[o] = float(betas[o])
    d.topq = topq
    return d


MODES = {"auto": 0, "dense": 1, "auto-exp": 2, "dense-exp": 3, "fp32": 4}


def predict_acquire(x_train, y_train, kinv, cands: CandidateSet, prior_mean, prior_variance,
                    length_scales, betas, *, outputs=("mu", "var", "acq"), topq=0,
                    excl_points=None, offset=0, count=None, out=None, device=None, mode="auto",
                    top_rec=None, prepare=False, float_type=None):
    """Score candidates [offset, offset+count) of `cands`.

    x_train [N, d], y_train [N or T, n_obj] (only the first N rows are read), kinv
    [n_obj, N, N] (invert_k output) -- device f64 tensors or arrays.  Returns a dict with
    the requested outputs (device tensors [n_obj, count] / [count]) and, if topq > 0,
    ``top_val`` / ``top_idx`` (device [topq]; index -1 = no candidate).  Asynchronous
    on the current stream.  mode "auto" computes the variance's quadratic form as
    q = 2 k^T (U k), U = upper triangle of (K^-1 + K^-T)/2 with the diagonal halved (the same
    form, half the matrix-core work, no factorisation); "dense" is update_variance's
    k^T (K^-1 k) verbatim.  The "-exp" modes disable the integer-grid
    separable K* generation (exp table) and evaluate every K* entry with exp().  "fp32" runs
    K* and the upper-form contraction in f32 on the f32 matrix cores (BASELINE config C5) and
    everything after the mean / quadratic form in f64.

    ``top_rec`` (optional f64 device tensor [2 topq]): the selection is written into it as one
    16-B-per-entry record block -- values in [:topq], int64 indices (bit pattern) in [topq:] --
    so that the multi-GPU exchange is ONE all_gather of it (distributed.exchange_topq_rec).
    A pinned host tensor is accepted too: the merge kernel then writes the selection straight
    into host memory (one shard: no device-to-host copy after the call).

    ``prepare=True`` returns a PreparedPredict instead of launching: calling it launches this
    call again (same buffers), without re-validating.

    ``float_type`` (default config.NUMBA_FLOAT_TYPE): np.float32 applies the reference's float32
    branch's variance floor MIN_VARIANCE = 1e-6 (config.py:57-61; BO_PREDICT_F32_FLOOR).
    """
    dev = require_device(device)
    x_train = as_dev(x_train, dev)
    y_train = as_dev(y_train, dev)
    kinv = as_dev(kinv, dev)
    n, n_obj = x_train.shape[0], len(prior_mean)
    if kinv.dim() != 3 or kinv.shape[0] != n_obj or kinv.shape[1] != kinv.shape[2] or kinv.shape[1] < n:
        raise ValueError("kinv must be [n_obj, >=N, >=N]")
    if y_train.shape[0] < n or y_train.shape[1] < n_obj:
        raise ValueError("y_train must be [>=N, n_obj]")
    if x_train.shape[1] != cands.dim:
        raise ValueError("x_train / candidate dimension mismatch")
    count = cands.n - offset if count is None else count
    if excl_points is not None:
        excl_points = as_dev(excl_points, dev)
    if not 0 <= topq <= _lib.MAX_TOPQ:
        raise ValueError(f"topq must be in [0, {_lib.MAX_TOPQ}]")
    desc = _fill_desc(x_train, y_train, kinv, cands, prior_mean, prior_variance, length_scales,
                      betas, offset, count, excl_points, topq)
    from .config import resolve_float_type
    desc.mode = MODES[mode] | (_lib.MODE_F32_FLOOR if resolve_float_type(float_type) == np.float32 else 0)
    res = {} if out is None else dict(out)
    for name in outputs:
        if name not in OUTPUT_NAMES:
            raise ValueError(f"unknown output {name}")
        if name not in res:
            shape = (count,) if name == "acq" else (n_obj, count)
            res[name] = torch.empty(shape, dtype=F64, device=dev)
    ld_out = None
    for name in ("mu", "var", "std_mu", "std_var", "ucb"):
        t = res.get(name)
        if t is not None:
            if t.dim() != 2 or t.shape[0] != n_obj or t.stride(1) != 1 or t.shape[1] < count:
                raise ValueError(f"{name} must be [n_obj, >=count] with unit column stride")
            if ld_out is not None and t.stride(0) != ld_out:
                raise ValueError("all per-objective outputs must share one row stride")
            ld_out = t.stride(0)
            setattr(desc, name, t.data_ptr())
    if res.get("acq") is not None:
        desc.acq = res["acq"].data_ptr()
    desc.ld_out = ld_out or count
    if topq:
        if top_rec is not None:
            on_dev = top_rec.device == dev or (top_rec.device.type == "cpu" and top_rec.is_pinned())
            if top_rec.dtype != F64 or top_rec.numel() != 2 * topq or not top_rec.is_contiguous() \
                    or not on_dev:
                raise ValueError("top_rec must be a contiguous f64 tensor of 2 * topq entries, on "
                                 "the device or in pinned host memory")
            res["top_val"] = top_rec[:topq]
            res["top_idx"] = top_rec[topq:].view(torch.int64)
        else:
            res["top_val"] = torch.empty(topq, dtype=F64, device=dev)
            res["top_idx"] = torch.empty(topq, dtype=torch.int64, device=dev)
        desc.top_val = res["top_val"].data_ptr()
        desc.top_idx = res["top_idx"].data_ptr()
    lib = _lib.load()
    nbytes = lib.bo_predict_workspace_size(desc)
    if nbytes == 0:
        raise _lib.BoNativeError(_lib.ERR_ARG, "bo_predict_workspace_size")
    ws = Workspace.get(nbytes, dev)
    # every raw pointer the descriptor (or a graph captured from it) holds must stay owned: the
    # inputs, the candidate set (its tensor, or the host Sobol descriptor read during the call)
    res["_keepalive"] = (x_train, y_train, kinv, excl_points, cands, cands.tensor, cands.sobol)
    call = PreparedPredict(lib, desc, ws, stream_handle(dev), res, dev)
    return call if prepare else call()


class PreparedPredict:
    """One validated bo_predict_acquire call (predict_acquire(..., prepare=True)): calling it
    re-launches the whole chain -- preparation (W packing, alpha, rows), the fused kernel and its
    in-kernel top-q merge -- on the same device buffers, which the caller may refill in place
    between calls.  Like a library plan object, it skips only the host-side validation and the
    descriptor build of predict_acquire (tens of microseconds of Python per call)."""

    def __init__(self, lib, desc, ws, stream, res, dev=None):
        self._lib, self._desc, self._ws, self._stream, self.res = lib, desc, ws, stream, res
        self._ws_ptr, self._ws_n = ws.data_ptr(), ws.numel()
        self._dev = dev

    def __call__(self):
        _lib.check(self._lib.bo_predict_acquire(self._desc, self._ws_ptr, self._ws_n, self._stream),
                   "bo_predict_acquire")
        return self.res

    def graphed(self):
        """The same call captured once as a HIP graph (preparation, fused kernel, merge): each
        replay is one graph launch from the host instead of three kernel launches, and the
        kernels start back to back.  Replays run on the current stream; the library's kernel
        timer (bo_profile_start/stop) does not see them."""
        dev = self._dev
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            _lib.check(self._lib.bo_predict_acquire(self._desc, self._ws_ptr, self._ws_n, side.cuda_stream),
                       "bo_predict_acquire")
            with torch.cuda.graph(g, stream=side, capture_error_mode="relaxed"):
                _lib.check(self._lib.bo_predict_acquire(self._desc, self._ws_ptr, self._ws_n,
                                                        side.cuda_stream), "bo_predict_acquire")
        torch.cuda.current_stream(dev).wait_stream(side)
        res = self.res

        def replay():
            g.replay()
            return res
        replay.graph = g
        # the graph bakes in the workspace pointer (packed W, partial lists) and the descriptor's
        # pointers: the replay owns this call (and through it the workspace tensor and res)
        replay.prepared = self
        return replay


def merge_topq(vals, idxs, q):
    """Host merge of per-shard top-q lists in the selection order of select_next_batch:
    NaN first, then descending value, ties by ascending global index; index -1 dropped."""
    vals = np.asarray(vals, dtype=np.float64).ravel()
    idxs = np.asarray(idxs, dtype=np.int64).ravel()
    keep = idxs >= 0
    vals, idxs = vals[keep], idxs[keep]
    nan = np.isnan(vals)
    order = np.lexsort((idxs, -np.where(nan, 0.0, vals), ~nan))
    return vals[order][:q], idxs[order][:q]
