"""Diagnostic: dump triangular-mode workspace (device Cholesky of K^-1, packed stream) and var."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np, torch
import bayesopt_smart_amd as bo
from bayesopt_smart_amd.device import Workspace
from conftest import predict_fixture
d = predict_fixture("g2_predict_512")
c = bo.CandidateSet.explicit(d["cand"])
out = {}
for mode in ("dense", "auto"):
    r = bo.predict_acquire(d["x"], d["y"], d["Kinv"], c, d["pm"], d["pv"], d["ls"], d["betas"],
                           outputs=("mu", "var", "acq"), topq=3, mode=mode)
    torch.cuda.synchronize()
    out["var_" + mode] = r["var"].cpu().numpy()
ws = Workspace._cache[("cuda", torch.cuda.current_device())]
out["ws_ptr"] = np.array([ws.data_ptr()])
out["ws"] = ws.cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/dbg_tri2.npz", **out)
print("saved", ws.numel())
