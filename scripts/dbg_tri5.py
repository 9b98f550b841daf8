"""Diagnostic (BO_ABL_DBGQ build): per-E-pair accumulators of tile 0 vs numpy R^T k."""
import sys, os, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
os.environ["BO_AMD_LIB"] = os.path.join(os.path.dirname(__file__), "..", "bayesopt_smart_amd", "libbo_amd_dbgq.so")
import numpy as np, torch
import bayesopt_smart_amd as bo
from conftest import predict_fixture
d = predict_fixture("g2_predict_512")
c = bo.CandidateSet.explicit(d["cand"])
L0 = bo._lib.load()
L0.bo_debug_set_tile(ctypes.c_longlong(int(os.environ.get("DBG_TILE", "0"))))
r = bo.predict_acquire(d["x"], d["y"], d["Kinv"], c, d["pm"], d["pv"], d["ls"], d["betas"],
                       outputs=("var",), mode="auto")
torch.cuda.synchronize()
L = bo._lib.load()
buf = np.zeros((64, 2, 4, 64))
L.bo_debug_dbgq.restype = ctypes.c_int
L.bo_debug_dbgq(buf.ctypes.data_as(ctypes.c_void_p))
np.savez("gpurun_out/dbgq.npz", buf=buf, var=r["var"].cpu().numpy())
print("ok")
