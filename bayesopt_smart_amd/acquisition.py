"""Drop-in mirror of bayesopt/acquisition.py on the MI355X (same names and semantics).

Arrays may be numpy (results copied back in place, as the reference mutates them) or HIP
device tensors.
"""

from __future__ import annotations

import ctypes as _C

import numpy as np
import torch

from . import _lib
from .device import F64, Workspace, require_device, stream_handle
from .kernels import _Arg, _dev_of, _host_vec

C_i64 = _C.c_int64


def upper_confidence_bound(mu, variance, beta):
    """acquisition.py:33-52 — mu + beta * sqrt(|variance|) (returns a new array)."""
    dev = _dev_of(mu, variance)
    m = _Arg(mu, dev)
    v = _Arg(variance, dev)
    out = torch.empty_like(m.t)
    _lib.check(_lib.load().bo_update_ucb(out.data_ptr(), m.ptr, v.ptr, 1, m.t.numel(),
                                         _host_vec([beta], 1), stream_handle(dev)), "bo_update_ucb")
    return out if isinstance(mu, torch.Tensor) else out.cpu().numpy()


def update_ucb(ucb, mu_objectives, variance_objectives, betas):
    """acquisition.py:55-81 — per-objective UCB, in place."""
    dev = _dev_of(ucb, mu_objectives)
    u = _Arg(ucb, dev, write=True)
    m = _Arg(mu_objectives, dev)
    v = _Arg(variance_objectives, dev)
    n_obj, n = m.t.shape
    _lib.check(_lib.load().bo_update_ucb(u.ptr, m.ptr, v.ptr, n_obj, n, _host_vec(betas, n_obj),
                                         stream_handle(dev)), "bo_update_ucb")
    u.finish()


def update_hypervolume_improvement(acquisition_values, ucb):
    """acquisition.py:89-108 — the reference's "HVI": sum of per-objective UCB, in place."""
    dev = _dev_of(acquisition_values, ucb)
    a = _Arg(acquisition_values, dev, write=True)
    u = _Arg(ucb, dev)
    n_obj, n = u.t.shape
    _lib.check(_lib.load().bo_update_hypervolume_improvement(a.ptr, u.ptr, n_obj, n, stream_handle(dev)),
               "bo_update_hypervolume_improvement")
    a.finish()


def _grid_args(cands):
    lo = (C_i64 * 8)(*(list(cands.lo or []) + [0] * (8 - len(cands.lo or []))))
    sh = (C_i64 * 8)(*(list(cands.shape or []) + [1] * (8 - len(cands.shape or []))))
    return lo, sh


class ExclusionMask:
    """The exclusion of acquisition.py:137-139 -- a candidate equal in every coordinate to an
    evaluated point is never selected -- as a device bit mask over one candidate shard
    ([offset, offset + count) of `cands`), kept across iterations (bo_excl_mask_update).

    The loop's evaluated set only grows (x_vector[:n], the new batch appended each iteration),
    so `update(points)` adds the rows it has not seen yet: one thread per new point on a grid,
    one pass over the shard otherwise.  A shorter or changed prefix rebuilds the mask.  The
    masked selections (bo_select_topq_masked, bo_hvi_select_topq_masked) then drop an excluded
    element as they load it: no per-call hash set and no probes."""

    def __init__(self, cands, offset=0, count=None, device=None):
        self.cands = cands
        self.offset = int(offset)
        self.count = int(cands.n - offset if count is None else count)
        self.dev = require_device(device)
        lib = _lib.load()
        self.bits = torch.zeros(lib.bo_excl_mask_bytes(self.count) // 4, dtype=torch.int32, device=self.dev)
        self.n_seen = 0
        self._seen = None              # host copy of the rows already in the mask

    @property
    def ptr(self):
        return self.bits.data_ptr()

    def update(self, evaluated_points):
        ev = np.ascontiguousarray(np.asarray(evaluated_points.cpu().numpy() if isinstance(evaluated_points, torch.Tensor)
                                             else evaluated_points, dtype=np.float64).reshape(-1, self.cands.dim))
        n = ev.shape[0]
        clear = n < self.n_seen or (self.n_seen > 0 and not np.array_equal(ev[: self.n_seen], self._seen))
        first = 0 if clear else self.n_seen
        if first == n and not clear:
            return self
        lib = _lib.load()
        ex = torch.as_tensor(ev, device=self.dev)
        ws = Workspace.get(lib.bo_excl_mask_workspace_size(n - first), self.dev)
        lo, sh = _grid_args(self.cands)
        carg = self.cands.cand_arg
        if self.cands.kind in ("i64", "f64"):
            carg = self.cands.tensor[self.offset:].data_ptr()
        _lib.check(lib.bo_excl_mask_update(self.ptr, self.count, self.cands.kind_code, carg, lo, sh,
                                           self.cands.dim, self.offset, ex.data_ptr() if n else None, first, n,
                                           1 if clear else 0, ws.data_ptr(), ws.numel(),
                                           stream_handle(self.dev)), "bo_excl_mask_update")
        self._keep = ex                # the points stay alive until the stream has used them
        self.n_seen = n
        self._seen = ev.copy()
        return self

    def excluded(self):
        """Host bool array [count]: the candidates the mask excludes."""
        w = self.bits.cpu().numpy().view(np.uint32)
        return np.unpackbits(w.view(np.uint8), bitorder="little")[: self.count].astype(bool)


def select_indices(acquisition_values, cands, evaluated_points, batch_size, dev=None, mask=None):
    """Global candidate indices of select_next_batch's choice (device top-q with exclusion).

    Order: NaN first, then descending value, ties by ascending index (the reference's
    argsort tie order is unspecified).  Batches above BO_MAX_TOPQ are taken in rounds,
    each round excluding the points already chosen.  `mask` (an ExclusionMask of the whole set,
    already updated with evaluated_points) replaces the per-call exclusion when the batch fits
    one call.
    """
    dev = dev or _dev_of(acquisition_values, evaluated_points)
    acq = _Arg(acquisition_values, dev)
    lib = _lib.load()
    if mask is not None and batch_size <= _lib.MAX_TOPQ:
        tv = torch.empty(batch_size, dtype=F64, device=dev)
        ti = torch.empty(batch_size, dtype=torch.int64, device=dev)
        ws = Workspace.get(lib.bo_select_topq_workspace_size(cands.n, batch_size), dev)
        _lib.check(lib.bo_select_topq_masked(acq.ptr, cands.n, 0, mask.ptr, batch_size, tv.data_ptr(),
                                             ti.data_ptr(), ws.data_ptr(), ws.numel(), stream_handle(dev)),
                   "bo_select_topq_masked")
        got = ti.cpu().numpy()
        return got[got >= 0].astype(np.int64)
    ev = np.asarray(evaluated_points.cpu().numpy() if isinstance(evaluated_points, torch.Tensor)
                    else evaluated_points, dtype=np.float64).reshape(-1, cands.dim)
    chosen = []
    while len(chosen) < batch_size:
        q = min(_lib.MAX_TOPQ, batch_size - len(chosen))
        excl = ev if not chosen else np.concatenate([ev, cands.points(np.array(chosen)).astype(np.float64)])
        ex = torch.as_tensor(np.ascontiguousarray(excl), device=dev)
        tv = torch.empty(q, dtype=F64, device=dev)
        ti = torch.empty(q, dtype=torch.int64, device=dev)
        lo, sh = _grid_args(cands)
        nbytes = lib.bo_select_topq_workspace_size(cands.n, q)
        ws = Workspace.get(nbytes, dev)
        _lib.check(lib.bo_select_topq(acq.ptr, cands.n, cands.kind_code, cands.cand_arg, lo, sh, cands.dim, 0, ex.data_ptr() if ex.numel() else None,
                                      ex.shape[0], q, tv.data_ptr(), ti.data_ptr(), ws.data_ptr(),
                                      ws.numel(), stream_handle(dev)), "bo_select_topq")
        got = [int(i) for i in ti.cpu().numpy() if i >= 0]
        chosen.extend(got)
        if len(got) < q:
            break
    return np.array(chosen, dtype=np.int64)


def select_next_batch(input_space, acquisition_values, evaluated_points, batch_size=3):
    """acquisition.py:116-144 — the best `batch_size` candidates (descending acquisition)
    that are not equal to an evaluated point; returns a new array of candidate rows."""
    from .predict import CandidateSet
    cands = CandidateSet.explicit(input_space, _dev_of(acquisition_values, input_space))
    idx = select_indices(acquisition_values, cands, evaluated_points, batch_size)
    if isinstance(input_space, torch.Tensor):
        return input_space[torch.as_tensor(idx, device=input_space.device)].cpu().numpy()
    return np.asarray(input_space)[idx]



# ------------------------------------------------------- exact hypervolume improvement
def hypervolume_boxes(front, reference_point) -> np.ndarray:
    """Disjoint boxes [lower, upper) (rows of 2*n_obj, upper may be +inf) covering the region
    above `reference_point` that no row of `front` dominates (maximisation); host decomposition
    in the library (bo_hvi_boxes).  Not in the reference (its reference point is unused,
    bayesian_optimization.py:65)."""
    f = np.ascontiguousarray(np.asarray(front.cpu().numpy() if isinstance(front, torch.Tensor) else front,
                                        dtype=np.float64))
    r = np.ascontiguousarray(np.asarray(reference_point, dtype=np.float64).ravel())
    n_obj = r.size
    f = f.reshape(-1, n_obj)
    lib = _lib.load()
    cnt = C_i64(0)
    dp = _C.POINTER(_C.c_double)
    cap = 1024
    while True:
        out = np.empty((cap, 2 * n_obj), dtype=np.float64)
        st = lib.bo_hvi_boxes(f.ctypes.data_as(dp), f.shape[0], n_obj, r.ctypes.data_as(dp),
                              out.ctypes.data, cap, _C.byref(cnt))
        if st == _lib.ERR_WORKSPACE and cnt.value > cap:   # retry with the reported count
            cap = int(cnt.value)
            continue
        _lib.check(st, "bo_hvi_boxes")
        return out[: cnt.value].copy()


def hypervolume_improvement_exact(ucb, front, reference_point, prior_mean, prior_variance, out=None):
    """Exact HVI of every candidate's UCB vector over `front`: acq = HV(front u {u}) - HV(front),
    u_k = prior_mean_k + sqrt(prior_variance_k) * ucb[k] (ucb: the reference's standardised
    per-objective UCB array, [n_obj, M], numpy or HIP tensor).  Returns acq ([M], a device
    tensor, or numpy for numpy `ucb`); written into `out` when given (in place)."""
    dev = _dev_of(out, ucb)
    u = _Arg(ucb, dev)
    n_obj, n = u.t.shape
    boxes = torch.as_tensor(hypervolume_boxes(front, reference_point), device=dev)
    acq = _Arg(out, dev, write=True) if out is not None else None
    dst = acq.t if acq is not None else torch.empty(n, dtype=F64, device=dev)
    pm = np.asarray(prior_mean, dtype=np.float64)[:n_obj]
    sc = np.sqrt(np.asarray(prior_variance, dtype=np.float64)[:n_obj])
    _lib.check(_lib.load().bo_hypervolume_improvement_exact(
        dst.data_ptr(), u.ptr, u.t.stride(0), n, n_obj, _host_vec(pm, n_obj), _host_vec(sc, n_obj),
        boxes.data_ptr() if boxes.numel() else None, boxes.shape[0], stream_handle(dev)),
        "bo_hypervolume_improvement_exact")
    if acq is not None:
        acq.finish()
        return out
    return dst if isinstance(ucb, torch.Tensor) else dst.cpu().numpy()


def hvi_select_indices(acquisition_values, ucb, y_vector, n_evaluations, reference_point, prior_mean,
                       prior_variance, cands, evaluated_points, batch_size, offset=0, return_record=False,
                       mask=None):
    """The exact-HVI acquisition AND its batch selection in one device pass (bo_hvi_select_topq,
    batch_size <= BO_MAX_TOPQ): acquisition_values (device, [count]) receives the HVI of the UCB
    vector of every candidate of the shard [offset, offset + count) over the Pareto front of
    y_vector[:n_evaluations]; returns the global indices of the shard's best batch_size candidates
    not equal to an evaluated point (select_next_batch's order) -- or, `return_record`, the device
    record block [2 batch_size] (values, bit-cast int64 indices) for the multi-rank exchange.
    `mask`: this shard's ExclusionMask (updated here with evaluated_points; only the new rows
    are added) -- the selection then runs bo_hvi_select_topq_masked."""
    from .pareto import is_pareto_efficient
    if batch_size > _lib.MAX_TOPQ:
        raise ValueError(f"hvi_select_indices handles batch_size <= {_lib.MAX_TOPQ}")
    y = y_vector[:n_evaluations]
    front = y[is_pareto_efficient(y)] if n_evaluations > 0 else np.zeros((0, len(reference_point)))
    if isinstance(front, torch.Tensor):
        front = front.cpu().numpy()
    dev = _dev_of(acquisition_values, ucb)
    u = _Arg(ucb, dev)
    acq = _Arg(acquisition_values, dev, write=True)
    n_obj, n = u.t.shape
    boxes = torch.as_tensor(hypervolume_boxes(front, reference_point), device=dev)
    rec = torch.empty(2 * batch_size, dtype=F64, device=dev)
    lib = _lib.load()
    ws = Workspace.get(lib.bo_select_topq_workspace_size(n, batch_size), dev)
    shift = _host_vec(prior_mean, n_obj)
    scale = _host_vec(np.sqrt(np.asarray(prior_variance, dtype=np.float64)), n_obj)
    if mask is not None:
        if mask.offset != offset or mask.count != n:
            raise ValueError("hvi_select_indices: the mask covers another shard")
        mask.update(evaluated_points)
        _lib.check(lib.bo_hvi_select_topq_masked(acq.ptr, u.ptr, u.t.stride(0), n, n_obj, shift, scale,
                                                 boxes.data_ptr() if boxes.numel() else None, boxes.shape[0],
                                                 offset, mask.ptr, batch_size, rec.data_ptr(),
                                                 rec.data_ptr() + 8 * batch_size, ws.data_ptr(), ws.numel(),
                                                 stream_handle(dev)), "bo_hvi_select_topq_masked")
    else:
        ev = np.asarray(evaluated_points.cpu().numpy() if isinstance(evaluated_points, torch.Tensor)
                        else evaluated_points, dtype=np.float64).reshape(-1, cands.dim)
        ex = torch.as_tensor(np.ascontiguousarray(ev), device=dev)
        lo, sh = _grid_args(cands)
        carg = cands.cand_arg
        if cands.kind in ("i64", "f64"):            # explicit candidates: the shard's rows
            carg = cands.tensor[offset:].data_ptr()
        _lib.check(lib.bo_hvi_select_topq(acq.ptr, u.ptr, u.t.stride(0), n, n_obj, shift, scale,
                                          boxes.data_ptr() if boxes.numel() else None, boxes.shape[0],
                                          cands.kind_code, carg, lo, sh, cands.dim, offset,
                                          ex.data_ptr() if ex.numel() else None, ex.shape[0], batch_size,
                                          rec.data_ptr(), rec.data_ptr() + 8 * batch_size, ws.data_ptr(),
                                          ws.numel(), stream_handle(dev)), "bo_hvi_select_topq")
    acq.finish()
    if return_record:
        return rec
    idx = rec[batch_size:].view(torch.int64).cpu().numpy()
    return idx[idx >= 0]


def update_hypervolume_improvement_exact(acquisition_values, ucb, y_vector, n_evaluations,
                                         reference_point, prior_mean, prior_variance):
    """The acquisition update of the loop (bayesian_optimization.py:195-199) as an exact HVI:
    the front is the Pareto-efficient subset (device filter, pareto.py:12-45) of the evaluated
    objectives y_vector[:n_evaluations]; in place into `acquisition_values`."""
    from .pareto import is_pareto_efficient
    y = y_vector[:n_evaluations]
    front = y[is_pareto_efficient(y)] if n_evaluations > 0 else np.zeros((0, len(reference_point)))
    if isinstance(front, torch.Tensor):
        front = front.cpu().numpy()
    hypervolume_improvement_exact(ucb, front, reference_point, prior_mean, prior_variance,
                                  out=acquisition_values)
