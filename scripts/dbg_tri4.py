"""Diagnostic: triangular path with dense random R^T restricted to one 32-row E-pair block."""
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
ls = d["ls"]
sq = ((x[:, None, :] - cand[None, :, :]) ** 2).sum(-1)
ks = np.exp(-0.5 * sq / ls[0] ** 2) * 1e3
rng = np.random.default_rng(0)
def run(W, tag):
    R = W.T
    kinv = np.stack([R @ R.T, R @ R.T])
    pv = 1e3
    e = ks / 1e3
    W = W * np.sqrt(0.25 * pv / (((W @ (pv * e)) ** 2).sum(0).max()))
    R = W.T
    kinv = np.stack([R @ R.T, R @ R.T])
    qt = ((W @ (pv * e)) ** 2).sum(0)
    out = []
    for mode in ("auto", "dense"):
        r = bo.predict_acquire(x, d["y"], kinv, c, d["pm"], [pv, pv], ls, d["betas"], outputs=("var",), mode=mode)
        torch.cuda.synchronize()
        qa = pv - r["var"].cpu().numpy()[0]
        err = np.abs(qa - qt) / qt.max()
        out.append((err.max(), int((err > 1e-9).sum())))
    print(tag, "auto/dense (max rel err, bad)", out, flush=True)
for ep in range(16):
    W = np.eye(n) * 1e-6
    rows = slice(32 * ep, 32 * ep + 32)
    blk = np.triu(rng.uniform(-1, 1, size=(n, n)) * 1e-2)
    W[rows] = blk[rows]
    W[np.arange(n), np.arange(n)] = np.where((np.arange(n) // 32) == ep, 1.0, 1e-6)
    run(W, f"ep {ep}")
W = np.triu(rng.uniform(-1, 1, size=(n, n)) * 1e-2) ; W[np.arange(n), np.arange(n)] = 1.0
run(W, "full")
