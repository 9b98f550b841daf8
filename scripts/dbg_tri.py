"""Diagnostic: triangular vs dense variance on the G2 golden (N=512), repeatability."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np, torch
import bayesopt_smart_amd as bo
from conftest import predict_fixture
d = predict_fixture("g2_predict_512")
c = bo.CandidateSet.explicit(d["cand"])
res = {}
for mode in ("dense", "auto", "auto", "auto"):
    r = bo.predict_acquire(d["x"], d["y"], d["Kinv"], c, d["pm"], d["pv"], d["ls"], d["betas"],
                           outputs=("mu", "var", "acq"), topq=3, mode=mode)
    torch.cuda.synchronize()
    v = r["var"].cpu().numpy()
    err = np.abs(v - d["var"]).max(axis=1) / d["pv"]
    print(mode, "max |dvar|/pv per obj", err, "top", r["top_idx"].cpu().numpy(), flush=True)
