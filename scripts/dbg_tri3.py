"""Diagnostic: probe the triangular variance path with crafted K^-1 = R R^T."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np, torch
import bayesopt_smart_amd as bo
from conftest import predict_fixture
d = predict_fixture("g2_predict_512")
c = bo.CandidateSet.explicit(d["cand"])
n = 512
x = d["x"]; cand = d["cand"].astype(float)
pv = np.array([1.0, 1.0]); ls = d["ls"]
sq = ((x[:, None, :] - cand[None, :, :]) ** 2).sum(-1)
ks = np.exp(-0.5 * sq / ls[0] ** 2)
def probe(R, tag):
    kinv = np.stack([R @ R.T, R @ R.T])
    r = bo.predict_acquire(x, d["y"], kinv, c, d["pm"], pv * 1e3, ls, d["betas"], outputs=("var",), mode="auto")
    r2 = bo.predict_acquire(x, d["y"], kinv, c, d["pm"], pv * 1e3, ls, d["betas"], outputs=("var",), mode="dense")
    torch.cuda.synchronize()
    qa = 1e3 - r["var"].cpu().numpy()[0]; qd = 1e3 - r2["var"].cpu().numpy()[0]
    qt = ((R.T @ (ks * 1e3)) ** 2).sum(0)
    print(tag, "auto err", np.abs(qa - qt).max() / 1e3, "dense err", np.abs(qd - qt).max() / 1e3, flush=True)
    return qa, qt
s = 1e-3 / 1.0
R = np.eye(n) * 1e-3 * 0.5
probe(R, "diag")
for (f, e) in [(5, 2), (40, 3), (100, 99), (300, 10), (431, 100), (480, 470), (510, 3), (510, 500), (511, 479), (479, 448)]:
    R2 = R.copy(); R2[f, e] = 0.4e-3
    qa, qt = probe(R2, f"R[{f},{e}]")
