"""bayesopt_smart_amd -- MI355X-native GP-predict + acquisition hot path of BayesOpt_smart.

Drop-in for the inner loop of alebal123bal/BayesOpt_smart
(bayesopt/bayesian_optimization.py:129-207): hand-written HIP/CDNA4 kernels behind a
C ABI (include/bo_amd.h), reached from Python through ctypes with PyTorch-ROCm tensors
as device memory.  Module layout mirrors the reference package:

  kernels.py               <- bayesopt/numba_kernels.py
  acquisition.py           <- bayesopt/acquisition.py
  pareto.py                <- bayesopt/pareto.py
  bayesian_optimization.py <- bayesopt/bayesian_optimization.py
  config.py                <- bayesopt/config.py
  predict.py               the fused hot path (no reference counterpart: the chain fused)
  distributed.py           candidate-shard parallelism (RCCL all_gather of top-q)
"""

__version__ = "0.1.0"

from . import _lib  # noqa: F401
from . import predict  # noqa: F401
from .predict import CandidateSet, merge_topq, predict_acquire  # noqa: F401


def __getattr__(name):
    # heavier modules import lazily (they pull in scipy)
    import importlib
    if name in ("kernels", "acquisition", "pareto", "bayesian_optimization", "config", "distributed"):
        return importlib.import_module(f".{name}", __name__)
    if name == "BayesianOptimization":
        return importlib.import_module(".bayesian_optimization", __name__).BayesianOptimization
    if name in ("is_pareto_efficient", "compute_pareto_front", "print_pareto_analysis"):
        return getattr(importlib.import_module(".pareto", __name__), name)
    if name == "select_next_batch":
        return importlib.import_module(".acquisition", __name__).select_next_batch
    raise AttributeError(name)
