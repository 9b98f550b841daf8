"""Constants mirrored from bayesopt/config.py (:28-90) and the orchestrator's defaults.  Like the
reference (config.py:22-25), importing this module seeds numpy's global RNG with RANDOM_SEED,
which makes the LHS initial design (numba_kernels.py:50-95) reproducible in exactly the
reference's (debug-mode) order.

Precision: the reference switches to float32 by editing NUMBA_FLOAT_TYPE (config.py:54), which
changes the jitters and the variance floor (:57-66) and the fit's optimiser to COBYLA
(numba_kernels.py:290-302).  Here the choice is made per call or per optimiser
(``float_type=np.float32``, or this module's NUMBA_FLOAT_TYPE, read at call time):
``precision_constants`` gives the branch's constants."""

import os

import numpy as np

DEBUG_MODE = os.environ.get("BAYESIAN_DEBUG", "False").lower() in ("true", "1", "yes")
RANDOM_SEED = 42
np.random.seed(RANDOM_SEED)

DEFAULT_PRIOR_MEAN = 0.0
DEFAULT_PRIOR_VARIANCE = 1.0
DEFAULT_LENGTH_SCALE = 1.0
DEFAULT_BETA = 1.0
DEFAULT_BATCH_SIZE = 3
DEFAULT_INITIAL_SAMPLES = 3

NUMBA_FLOAT_TYPE = np.float64


def resolve_float_type(float_type=None):
    """np.float32 or np.float64 from a dtype / name ('float32', 'fp32', 'f32', ...); None = this
    module's NUMBA_FLOAT_TYPE at call time."""
    ft = NUMBA_FLOAT_TYPE if float_type is None else float_type
    if isinstance(ft, str):
        ft = {"float32": np.float32, "fp32": np.float32, "f32": np.float32,
              "float64": np.float64, "fp64": np.float64, "f64": np.float64}.get(ft.lower(), ft)
    ft = np.dtype(ft).type
    if ft not in (np.float32, np.float64):
        raise ValueError(f"float_type must be float32 or float64 (got {float_type!r})")
    return ft


def precision_constants(float_type=None):
    """(KERNEL_JITTER, CHOLESKY_JITTER, MIN_VARIANCE) of the reference's branch (config.py:57-66)."""
    if resolve_float_type(float_type) == np.float32:
        return 1e-3, 1e-4, 1e-6
    return 1e-6, 1e-8, 1e-10


KERNEL_JITTER, CHOLESKY_JITTER, MIN_VARIANCE = precision_constants(NUMBA_FLOAT_TYPE)

HYPERPARAM_METHOD = "Powell"
HYPERPARAM_XTOL = 1e-3
HYPERPARAM_FTOL = 1e-4
HYPERPARAM_MAXITER = 1000
HYPERPARAM_MIN_BOUND = 1e-5

DEFAULT_PLOT_ENABLED = True
