"""Build libbo_amd.so in-tree with hipcc for gfx950 (no torch involvement).

    python -m bayesopt_smart_amd.csrc.build        # or via __graft_entry__.build()

Objects are cached by source mtime under csrc/build/; `-j` parallel compiles.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
VARIANT = os.environ.get("BO_BUILD_VARIANT", "")      # diagnostic builds: -DBO_ABL_<name>
LIB = os.path.join(PKG, f"libbo_amd{('_' + VARIANT.lower().replace(',', '_')) if VARIANT else ''}.so")
BUILD = os.path.join(HERE, "build" + (("_" + VARIANT.lower()) if VARIANT else ""))
SOURCES = ["bo_predict_d2.hip", "bo_predict_d4.hip", "bo_predict_d6.hip", "bo_predict_d8.hip",
           "bo_predict_s2.hip", "bo_predict_s4.hip", "bo_predict_s6.hip", "bo_predict_s8.hip",
           "bo_predict.hip", "bo_fit.hip", "bo_lu.hip", "bo_select.hip", "bo_misc.hip", "bo_hvi.hip",
           "bo_powell.hip"]
HEADERS = ["bo_common.h", "bo_predict_impl.h", os.path.join("..", "..", "include", "bo_amd.h")]
ARCH = os.environ.get("BO_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-I", os.path.join(ROOT, "include")] + \
        [(f"-DBO_{v[4:]}" if v.startswith("DEF_") else f"-DBO_ABL_{v}") for v in VARIANT.split(",") if v] + \
        os.environ.get("BO_EXTRA_FLAGS", "").split()   # diagnostic builds (with a VARIANT name)


# per-source flags: the small-N predict kernels keep their MFMA accumulators in arch VGPRs; the
# 2-D translation units (the integer-grid configs C2/C3) use the max-ILP machine scheduler
# (same-box A/B: C2 -1.5 %, C3 -0.5 %; on the 6-D Sobol kernel of C4 it measured +4.5 %)
EXTRA = {f"bo_predict_s{d}.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"] for d in (2, 4, 6, 8)}
for _src in ("bo_predict_d2.hip", "bo_predict_s2.hip"):
    EXTRA[_src] = EXTRA.get(_src, []) + ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]


def _hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _newest_header():
    return max(os.path.getmtime(os.path.join(HERE, h)) for h in HEADERS)


def _compile(src, hdr_mtime):
    s = os.path.join(HERE, src)
    o = os.path.join(BUILD, src + ".o")
    if os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(s), hdr_mtime):
        return o, False
    cmd = [_hipcc(), *FLAGS, *EXTRA.get(src, []), "-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return o, True


def build(verbose=True, jobs=None):
    os.makedirs(BUILD, exist_ok=True)
    hdr = _newest_header()
    jobs = jobs or min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, hdr), SOURCES))
    objs = [o for o, _ in results]
    rebuilt = any(r for _, r in results)
    if rebuilt or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB + ".tmp"      # linked aside, then renamed: a reader never sees a partial file
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
