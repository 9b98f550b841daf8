"""Phase breakdown of the fused kernel from the BO_ABL_STAMPS diagnostic build."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["BO_AMD_LIB"] = os.path.join(ROOT, "bayesopt_smart_amd", "libbo_amd_stamps.so")
import bench  # noqa: E402
import bayesopt_smart_amd as bo  # noqa: E402

x, y, pm, pv, ls, betas, kinv, rows = bench.make_problem(1)
c = bo.CandidateSet.grid([(0, 1024), (0, 1024)])
xd, yd, kd = (torch.tensor(a, device="cuda") for a in (x, y, kinv))
L = bo._lib.load()
for mode in sys.argv[1:] or ["auto"]:
    bo.predict_acquire(xd, yd, kd, c, pm, pv, ls, betas, outputs=("acq",), topq=3, mode=mode)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (4096 * 8))()
    fn = L.bo_debug_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn(buf, 4096)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8)
    a = a[a[:, 4] > 0][:, :4].astype(np.float64)
    names = ["setup+row pass", "chunk loop", "epilogue q", "outputs/topq/rest"]
    tot = a.sum(1).mean()
    print(mode, "waves", a.shape[0], "cycles/wave", f"{tot:.4g}",
          {n: f"{v / tot * 100:.1f}%" for n, v in zip(names, a.mean(0))})
