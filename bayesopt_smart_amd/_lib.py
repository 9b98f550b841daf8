"""ctypes binding of libbo_amd.so (include/bo_amd.h).

The product path has no CPU fallback: if the library or a HIP device is missing the
calls raise ``BoNativeError`` / ``RuntimeError``.  Error statuses of the fit entry
points map to ``numpy.linalg.LinAlgError`` exactly like the reference's LAPACK calls
(bayesopt/numba_kernels.py:214, :401).
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BO_AMD_LIB", os.path.join(_HERE, "libbo_amd.so"))

MAX_OBJ = 8
MAX_DIM = 8
MAX_TOPQ = 48

OK, ERR_ARG, ERR_UNSUPPORTED, ERR_WORKSPACE, ERR_HIP, ERR_NOT_PD, ERR_SINGULAR = range(7)
CAND_I64, CAND_F64, CAND_GRID, CAND_SOBOL = 0, 1, 2, 3
ABI_VERSION = 5
MODE_AUTO, MODE_DENSE, MODE_NO_SEPARABLE, MODE_FP32, MODE_F32_FLOOR = 0, 1, 2, 4, 8

c_dbl_p = C.POINTER(C.c_double)
c_vp = C.c_void_p


class BoNativeError(RuntimeError):
    def __init__(self, status, what):
        self.status = status
        super().__init__(f"{what}: {status_string(status)} (status {status})")


class PredictDesc(C.Structure):
    """Mirror of bo_predict_desc (include/bo_amd.h)."""

    _fields_ = [
        ("n_obj", C.c_int32), ("dim", C.c_int32), ("n_train", C.c_int64),
        ("x_train", c_vp), ("y_train", c_vp), ("ld_y", C.c_int64),
        ("kinv", c_vp), ("ld_k", C.c_int64),
        ("cand_kind", C.c_int32), ("mode", C.c_int32),
        ("cand", c_vp), ("n_cand", C.c_int64), ("cand_offset", C.c_int64),
        ("grid_lo", C.c_int64 * MAX_DIM), ("grid_shape", C.c_int64 * MAX_DIM),
        ("excl_points", c_vp), ("n_excl", C.c_int64),
        ("prior_mean", C.c_double * MAX_OBJ), ("prior_var", C.c_double * MAX_OBJ),
        ("length_scale", C.c_double * MAX_OBJ), ("beta", C.c_double * MAX_OBJ),
        ("mu", c_vp), ("var", c_vp), ("std_mu", c_vp), ("std_var", c_vp),
        ("ucb", c_vp), ("acq", c_vp), ("ld_out", C.c_int64),
        ("topq", C.c_int32), ("reserved1", C.c_int32),
        ("top_val", c_vp), ("top_idx", c_vp),
    ]


class PowellResult(C.Structure):
    """Mirror of bo_powell_result (include/bo_amd.h)."""

    _fields_ = [("fun", C.c_double), ("nfev", C.c_int64), ("nit", C.c_int64),
                ("device_calls", C.c_int64), ("warnflag", C.c_int32), ("reserved", C.c_int32)]


# int (*)(const double* x, int32_t n, double* f, void* user)
OBJECTIVE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_double), C.c_void_p)
# double (*)(double x, int32_t which): tan (0) / atan (1)
TRIG_FN = C.CFUNCTYPE(C.c_double, C.c_double, C.c_int32)


def _numpy_trig(x, which):
    import numpy
    return float(numpy.tan(numpy.float64(x)) if which == 0 else numpy.arctan(numpy.float64(x)))


NUMPY_TRIG = TRIG_FN(_numpy_trig)    # numpy's tan/atan: scipy's evaluation points bit for bit


class SobolDesc(C.Structure):
    """Mirror of bo_sobol_desc (include/bo_amd.h)."""

    _fields_ = [("bits", C.c_int32), ("reserved", C.c_int32),
                ("lo", C.c_double * MAX_DIM), ("scale", C.c_double * MAX_DIM)]


_SIGS = {
    "bo_abi_version": (C.c_int, []),
    "bo_status_string": (C.c_char_p, [C.c_int]),
    "bo_device_count": (C.c_int, []),
    "bo_predict_workspace_size": (C.c_size_t, [C.POINTER(PredictDesc)]),
    "bo_predict_acquire": (C.c_int, [C.POINTER(PredictDesc), c_vp, C.c_size_t, c_vp]),
    "bo_update_k": (C.c_int, [c_vp, C.c_int64, C.c_int32, c_vp, C.c_int32, C.c_int64, C.c_int64,
                              c_dbl_p, c_dbl_p, c_vp]),
    "bo_update_k_star": (C.c_int, [c_vp, C.c_int64, C.c_int32, c_vp, C.c_int32, C.c_int32, c_vp,
                                   C.c_int64, C.c_int64, C.c_int64, c_dbl_p, c_dbl_p, c_vp]),
    "bo_update_mean_variance": (C.c_int, [c_vp, c_vp, c_vp, C.c_int64, C.c_int32, C.c_int64, c_vp,
                                          C.c_int64, c_vp, C.c_int64, C.c_int64, c_dbl_p, c_dbl_p,
                                          c_vp, C.c_size_t, c_vp]),
    "bo_update_mean_variance_workspace_size": (C.c_size_t, [C.c_int32, C.c_int64]),
    "bo_standardize_ucb_hvi": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C.c_int32, C.c_int64,
                                         c_dbl_p, c_dbl_p, c_dbl_p, c_vp]),
    "bo_update_ucb": (C.c_int, [c_vp, c_vp, c_vp, C.c_int32, C.c_int64, c_dbl_p, c_vp]),
    "bo_update_hypervolume_improvement": (C.c_int, [c_vp, c_vp, C.c_int32, C.c_int64, c_vp]),
    "bo_select_topq": (C.c_int, [c_vp, C.c_int64, C.c_int32, c_vp, C.POINTER(C.c_int64),
                                 C.POINTER(C.c_int64), C.c_int32, C.c_int64, c_vp, C.c_int64,
                                 C.c_int32, c_vp, c_vp, c_vp, C.c_size_t, c_vp]),
    "bo_select_topq_workspace_size": (C.c_size_t, [C.c_int64, C.c_int32]),
    "bo_excl_mask_bytes": (C.c_size_t, [C.c_int64]),
    "bo_excl_mask_workspace_size": (C.c_size_t, [C.c_int64]),
    "bo_excl_mask_update": (C.c_int, [c_vp, C.c_int64, C.c_int32, c_vp, C.POINTER(C.c_int64),
                                      C.POINTER(C.c_int64), C.c_int32, C.c_int64, c_vp, C.c_int64,
                                      C.c_int64, C.c_int32, c_vp, C.c_size_t, c_vp]),
    "bo_select_topq_masked": (C.c_int, [c_vp, C.c_int64, C.c_int64, c_vp, C.c_int32, c_vp, c_vp, c_vp,
                                        C.c_size_t, c_vp]),
    "bo_hvi_select_topq_masked": (C.c_int, [c_vp, c_vp, C.c_int64, C.c_int64, C.c_int32, c_dbl_p, c_dbl_p,
                                            c_vp, C.c_int64, C.c_int64, c_vp, C.c_int32, c_vp, c_vp, c_vp,
                                            C.c_size_t, c_vp]),
    "bo_pareto_mask": (C.c_int, [c_vp, C.c_int64, C.c_int32, c_vp, c_vp]),
    "bo_hvi_boxes": (C.c_int, [c_dbl_p, C.c_int64, C.c_int32, c_dbl_p, c_vp, C.c_int64,
                               C.POINTER(C.c_int64)]),
    "bo_hypervolume_improvement_exact": (C.c_int, [c_vp, c_vp, C.c_int64, C.c_int64, C.c_int32,
                                                   c_dbl_p, c_dbl_p, c_vp, C.c_int64, c_vp]),
    "bo_hvi_select_topq": (C.c_int, [c_vp, c_vp, C.c_int64, C.c_int64, C.c_int32, c_dbl_p, c_dbl_p, c_vp,
                                     C.c_int64, C.c_int32, c_vp, C.POINTER(C.c_int64),
                                     C.POINTER(C.c_int64), C.c_int32, C.c_int64, c_vp, C.c_int64,
                                     C.c_int32, c_vp, c_vp, c_vp, C.c_size_t, c_vp]),
    "bo_box_volume_sum": (C.c_int, [c_vp, C.c_int64, C.c_int32, c_dbl_p, c_vp, c_vp]),
    "bo_invert_k": (C.c_int, [c_vp, c_vp, C.c_int64, C.c_int32, C.c_int64, c_vp, C.c_size_t, c_vp]),
    "bo_invert_k_workspace_size": (C.c_size_t, [C.c_int32, C.c_int64]),
    "bo_invert_k_jitter": (C.c_int, [c_vp, c_vp, C.c_int64, C.c_int32, C.c_int64, C.c_double, c_vp,
                                     C.c_size_t, c_vp]),
    "bo_invert_k_ex": (C.c_int, [c_vp, c_vp, C.c_int64, C.c_int32, C.c_int64, C.c_double,
                                 C.POINTER(C.c_int32), C.POINTER(C.c_int32), c_vp, C.c_size_t, c_vp]),
    "bo_compute_mll_each_jitter": (C.c_int, [c_dbl_p, c_vp, C.c_int32, c_vp, C.c_int64, c_vp, C.c_int64,
                                             C.c_int32, c_dbl_p, c_dbl_p, c_dbl_p, C.c_int64, C.c_double,
                                             c_vp, C.c_size_t, c_vp]),
    "bo_powell_minimize": (C.c_int, [OBJECTIVE_FN, c_vp, c_dbl_p, C.c_int32, c_dbl_p, c_dbl_p, C.c_double,
                                     C.c_double, C.c_int64, C.c_int64, TRIG_FN, c_dbl_p, C.POINTER(PowellResult)]),
    "bo_optimize_hyperparams_mll": (C.c_int, [c_vp, C.c_int32, c_vp, C.c_int64, c_vp, C.c_int64, C.c_int32,
                                              c_dbl_p, c_dbl_p, c_dbl_p, C.c_int64, C.c_double, C.c_double,
                                              C.c_double, C.c_int64, C.c_double, TRIG_FN, c_vp, C.c_size_t, c_vp,
                                              C.POINTER(PowellResult), c_dbl_p]),
    "bo_invert_k_path_counts": (C.c_int, [C.POINTER(C.c_int64)]),
    "bo_fit_path_counts": (C.c_int, [C.POINTER(C.c_int64)]),
    "bo_compute_mll": (C.c_int, [c_dbl_p, c_vp, C.c_int32, c_vp, C.c_int64, c_vp, C.c_int64,
                                 C.c_int32, c_dbl_p, c_dbl_p, c_dbl_p, C.c_int64, c_vp, C.c_size_t,
                                 c_vp]),
    "bo_compute_mll_workspace_size": (C.c_size_t, [C.c_int32, C.c_int64]),
    "bo_compute_mll_each": (C.c_int, [c_dbl_p, c_vp, C.c_int32, c_vp, C.c_int64, c_vp, C.c_int64,
                                      C.c_int32, c_dbl_p, c_dbl_p, c_dbl_p, C.c_int64, c_vp, C.c_size_t,
                                      c_vp]),
    "bo_sobol_points": (C.c_int, [C.POINTER(SobolDesc), C.c_int32, C.POINTER(C.c_int64), C.c_int64,
                                  c_dbl_p]),
    "bo_sobol_direction_numbers": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(C.c_uint32)]),
    "bo_selftest_mfma_f64": (C.c_int, [c_vp, c_vp, c_vp, c_vp]),
    "bo_selftest_mfma_f32": (C.c_int, [c_vp, c_vp, c_vp, c_vp]),
    "bo_profile_start": (C.c_int, [C.c_int]),
    "bo_profile_stop": (C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_int)]),
}

_lib = None


def load():
    """Load libbo_amd.so and declare every exported symbol (raises if missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BoNativeError(ERR_UNSUPPORTED,
                            f"{LIB_PATH} not built (run __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.bo_abi_version() != ABI_VERSION:
        raise BoNativeError(ERR_UNSUPPORTED, "ABI version mismatch")
    _lib = lib
    return lib


def symbols():
    return list(_SIGS)


def status_string(status):
    try:
        return load().bo_status_string(int(status)).decode()
    except Exception:  # pragma: no cover - only used while formatting an error
        return "unknown"


def check(status, what):
    if status == OK:
        return
    if status in (ERR_NOT_PD, ERR_SINGULAR):
        raise np.linalg.LinAlgError(status_string(status))
    raise BoNativeError(status, what)


def invert_k_path_counts():
    """{'cholesky', 'lu', 'gauss_jordan'}: per-objective counts of bo_invert_k's paths so far."""
    arr = (C.c_int64 * 3)()
    check(load().bo_invert_k_path_counts(arr), "bo_invert_k_path_counts")
    return {"cholesky": arr[0], "lu": arr[1], "gauss_jordan": arr[2]}


def fit_path_counts():
    """{'persistent', 'launches', 'aborted'}: how the factorisations so far were scheduled."""
    arr = (C.c_int64 * 3)()
    check(load().bo_fit_path_counts(arr), "bo_fit_path_counts")
    return {"persistent": arr[0], "launches": arr[1], "aborted": arr[2]}


def dbl_array(values, n=None):
    vals = [float(v) for v in values]
    n = n or len(vals)
    arr = (C.c_double * max(n, 1))(*vals)
    return arr
