"""Full-size CPU reference arrays for the -m gpu parity tests.

Every candidate of a BASELINE config (C2 262,144 / C3 1,048,576 / C4 2,097,152 / C5's 2^18
prefix and its 8-GPU shards 0 and 7, 524,288 each) is scored by oracle/cpu_ref.c -- the C/OpenMP restatement of the reference chain
update_k_star -> update_mean -> update_variance -> standardize_objectives -> update_ucb ->
update_hypervolume_improvement (bayesopt/numba_kernels.py:406-570, bayesopt/acquisition.py:33-108),
pinned to the reference's own outputs by tests/test_oracle_golden.py::test_cpu_ref_matches_oracle.
The GPU arrays are then compared value by value (SURVEY.md §8c tolerances, tests/parity.py) and
the GPU's top-q selection is judged against the CPU acquisition array, not the GPU's own.

Results are cached per problem key so the parametrised modes of one config score it once.
TEST INFRASTRUCTURE ONLY.
"""

import numpy as np

_CACHE = {}


def cpu_full(key, x, y, cand, kinv, pm, pv, ls, betas):
    """mu, var, ucb, acq of every row of `cand` (f64 [M, d]) on the host cores."""
    if key not in _CACHE:
        from oracle import cpu_ref
        _CACHE[key] = cpu_ref.predict_acquire(x, y, np.asarray(cand, dtype=np.float64), kinv, pm, pv,
                                              ls, betas, ucb=True)
    return _CACHE[key]


def grid_points_2d(rows, side):
    """The reference's 'ij' meshgrid input_space (bayesian_optimization.py:338-340), f64."""
    lin = np.arange(rows * side, dtype=np.int64)
    return np.stack([lin // side, lin % side], axis=1).astype(np.float64)
