"""Constants mirrored from bayesopt/config.py (fp64 branch, :57-66) and the orchestrator's
defaults (:28-49).  Like the reference (config.py:22-25), importing this module seeds numpy's
global RNG with RANDOM_SEED, which makes the LHS initial design (numba_kernels.py:50-95)
reproducible in exactly the reference's (debug-mode) order."""

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
KERNEL_JITTER = 1e-6
CHOLESKY_JITTER = 1e-8
MIN_VARIANCE = 1e-10

HYPERPARAM_METHOD = "Powell"
HYPERPARAM_XTOL = 1e-3
HYPERPARAM_FTOL = 1e-4
HYPERPARAM_MAXITER = 1000
HYPERPARAM_MIN_BOUND = 1e-5

DEFAULT_PLOT_ENABLED = True
