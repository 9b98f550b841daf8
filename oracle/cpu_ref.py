"""ctypes binding of oracle/cpu_ref.c (the C/OpenMP restatement of the reference chain).

TEST / MEASUREMENT INFRASTRUCTURE ONLY: used by tests/ (pinned against oracle_np) and by
bench.py's cpu_baseline leg; never by bayesopt_smart_amd.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpu_ref.c")
# BO_CPU_REF_LIB: another build of the same source (scripts/host_sanitize.sh's ASan/UBSan build)
LIB = os.environ.get("BO_CPU_REF_LIB", os.path.join(HERE, "libcpu_ref.so"))
# portable x86-64 (AVX2 + FMA): the GPU box's host CPU is not this container's
FLAGS = ["-O3", "-march=x86-64-v3", "-fopenmp", "-shared", "-fPIC"]

_lib = None


def build():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.run(["gcc", *FLAGS, SRC, "-o", LIB, "-lm"], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        P = C.c_void_p
        lib.bo_cpu_predict_acquire.argtypes = [C.c_int, C.c_int, C.c_int, P, P, P, C.c_long, P, P, P,
                                               P, P, P, P, P, P, C.c_int]
        lib.bo_cpu_predict_acquire.restype = C.c_int
        lib.bo_cpu_select.argtypes = [P, P, C.c_long, C.c_int, P, C.c_long, C.c_int, P]
        lib.bo_cpu_select.restype = C.c_int
        lib.bo_cpu_set_dgemm.argtypes = [P]
        lib.bo_cpu_has_dgemm.restype = C.c_int
        _install_system_dgemm(lib)
        _lib = lib
    return _lib


_blas = None


def _install_system_dgemm(lib):
    """Point cpu_ref.c at numpy's bundled OpenBLAS cblas_dgemm (64-bit ints) -- the system DGEMM
    the reference's np.dot runs on -- when it can be found; else the built-in AVX2 loop."""
    global _blas
    import glob
    import numpy
    libdir = os.path.join(os.path.dirname(numpy.__file__), "..", "numpy.libs")
    for path in sorted(glob.glob(os.path.join(libdir, "libscipy_openblas64_*.so"))):
        try:
            b = C.CDLL(path)
            fn = b.scipy_cblas_dgemm64_
        except (OSError, AttributeError):
            continue
        b.scipy_openblas_set_num_threads64_.argtypes = [C.c_int]
        b.scipy_openblas_get_num_threads64_.restype = C.c_int
        lib.bo_cpu_set_dgemm(C.cast(fn, C.c_void_p))
        _blas = b
        return
    lib.bo_cpu_set_dgemm(None)


def dgemm_name():
    load()
    return "OpenBLAS cblas_dgemm (numpy's scipy-openblas64)" if _blas is not None else \
        "built-in AVX2 register-tiled loop"


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def predict_acquire(x, y, cand, kinv, pm, pv, ls, betas, threads=None, outputs=True, ucb=False):
    """mu, var (optional), ucb (optional) and acq over `cand` (f64 [M, d]) with the reference's
    algorithm."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    n, d = x.shape
    n_obj = len(pm)
    y = np.ascontiguousarray(np.asarray(y, dtype=np.float64)[:n, :n_obj])
    cand = np.ascontiguousarray(cand, dtype=np.float64)
    m = cand.shape[0]
    kinv = np.ascontiguousarray(np.asarray(kinv, dtype=np.float64)[:, :n, :n])
    vec = lambda v: np.ascontiguousarray(np.asarray(v, dtype=np.float64)[:n_obj])  # noqa: E731
    mu = np.empty((n_obj, m)) if outputs else None
    var = np.empty((n_obj, m)) if outputs else None
    ucb_a = np.empty((n_obj, m)) if ucb else None
    acq = np.empty(m)
    threads = threads or int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    lib = load()
    # one single-threaded DGEMM per OpenMP thread and candidate block (no nested BLAS threads)
    nt = _blas.scipy_openblas_get_num_threads64_() if _blas is not None else 0
    if _blas is not None:
        _blas.scipy_openblas_set_num_threads64_(1)
    try:
        lib.bo_cpu_predict_acquire(n, d, n_obj, _p(x), _p(y), _p(cand), m, _p(kinv), _p(vec(pm)),
                                   _p(vec(pv)), _p(vec(ls)), _p(vec(betas)), _p(mu), _p(var),
                                   _p(ucb_a), _p(acq), threads)
    finally:
        if _blas is not None:
            _blas.scipy_openblas_set_num_threads64_(nt)
    out = {"mu": mu, "var": var, "acq": acq}
    if ucb:
        out["ucb"] = ucb_a
    return out


def select(acq, cand, excl, q):
    """Candidate indices of select_next_batch's choice (descending, evaluated points skipped)."""
    acq = np.ascontiguousarray(acq, dtype=np.float64)
    cand = np.ascontiguousarray(cand, dtype=np.float64)
    excl = np.ascontiguousarray(excl, dtype=np.float64).reshape(-1, cand.shape[1])
    out = np.empty(q, dtype=np.int64)
    load().bo_cpu_select(_p(acq), _p(cand), cand.shape[0], cand.shape[1], _p(excl), excl.shape[0], q,
                         _p(out))
    return out
