"""Drop-in mirror of bayesopt/pareto.py: the non-dominated filter runs on the device
(bo_pareto_mask, bit-exact comparisons)."""

from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from . import _lib
from .device import stream_handle
from .kernels import _Arg, _dev_of


def is_pareto_efficient(y_vector) -> np.ndarray:
    """pareto.py:12-45 — boolean mask of the points no other point dominates (maximisation)."""
    dev = _dev_of(y_vector)
    y = _Arg(y_vector, dev)
    n = y.t.shape[0]
    n_obj = y.t.shape[1] if y.t.dim() == 2 else 1
    mask = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _lib.check(_lib.load().bo_pareto_mask(y.ptr, n, n_obj, mask.data_ptr(), stream_handle(dev)),
               "bo_pareto_mask")
    return mask[:n].cpu().numpy().astype(bool)


def compute_pareto_front(x_vector, y_vector) -> Tuple[np.ndarray, np.ndarray]:
    """pareto.py:48-64."""
    m = is_pareto_efficient(y_vector)
    x = x_vector.cpu().numpy() if isinstance(x_vector, torch.Tensor) else np.asarray(x_vector)
    y = y_vector.cpu().numpy() if isinstance(y_vector, torch.Tensor) else np.asarray(y_vector)
    return x[m], y[m]


def print_pareto_analysis(pareto_inputs, pareto_objectives) -> None:
    """pareto.py:67-80."""
    print("📊 Pareto Analysis Results:")
    for i, (inp, obj) in enumerate(zip(pareto_inputs, pareto_objectives)):
        print(f"Input: {inp}, Pareto Point {i + 1}: {obj}")
