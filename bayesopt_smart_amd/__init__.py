"""bayesopt_smart_amd -- MI355X-native GP-predict + acquisition hot path of BayesOpt_smart.

Drop-in for the inner loop of alebal123bal/BayesOpt_smart
(bayesopt/bayesian_optimization.py:129-207): hand-written HIP/CDNA4 kernels behind a
C ABI (include/bo_amd.h), reached from Python through ctypes with PyTorch-ROCm tensors
as device memory.  See DESIGN.md.
"""

__version__ = "0.1.0"

from . import _lib  # noqa: F401
from . import predict  # noqa: F401
from .predict import CandidateSet, predict_acquire, merge_topq  # noqa: F401
