"""Host time of the drop-in loop's acquisition call (DeviceBackend.select ->
sharded_predict_acquire -> predict_acquire -> bo_predict_acquire), split into its Python and
library parts, at the C3 loop's N; the kernels themselves are asynchronous, so the host times are
those of the calls returning (launch-side cost), then the synchronisation."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import bayesopt_smart_amd as bo  # noqa: E402
from bayesopt_smart_amd.bayesian_optimization import DeviceBackend  # noqa: E402

cfg = bench.CONFIGS["C3"]
x, y, pm, pv, ls, betas, _, cand = bench.make_config_problem(cfg, 1)
dev = torch.device("cuda", 0)
cands = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])])
n = 515
rng = np.random.default_rng(5)
extra = rng.choice(1024 * 1024, size=n - x.shape[0], replace=False)
xe = np.concatenate([x, np.stack([extra // 1024, extra % 1024], 1).astype(np.float64)])
ye = bench.toy_function(xe)
be = DeviceBackend(cands, 2, 600, dev)
lsv = np.full(2, 680.0)
xd, yd = torch.tensor(xe, device=dev), torch.tensor(ye, device=dev)
bo.kernels.update_k(be.bufs.kernel_matrices, xd, 0, n, pv, lsv)
kinv = bo.kernels.invert_k(n, be.bufs.kernel_matrices, lu_hint=[True, True])
torch.cuda.synchronize()
fitted = (xd, yd, kinv)
for rep in range(4):
    t0 = time.perf_counter()
    idx = be.select(fitted, pm, pv, lsv, betas, 3, xe)
    t1 = time.perf_counter()
    out = be._outputs()
    t2 = time.perf_counter()
    r = bo.predict_acquire(xd, yd, kinv, cands, pm, pv, lsv, betas, outputs=tuple(out), topq=3, out=out, device=dev)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    prep = bo.predict_acquire(xd, yd, kinv, cands, pm, pv, lsv, betas, outputs=tuple(out), topq=3, out=out,
                              device=dev, prepare=True)
    t5 = time.perf_counter()
    prep()
    t6 = time.perf_counter()
    torch.cuda.synchronize()
    t7 = time.perf_counter()
    print(f"select (sync'd by its .cpu()) {1e3*(t1-t0):.3f} ms | predict_acquire call returns {1e3*(t3-t2):.3f} ms, "
          f"sync {1e3*(t4-t3):.3f} | prepare {1e3*(t5-t4):.3f} ms, prepared call returns {1e3*(t6-t5):.3f} ms, "
          f"sync {1e3*(t7-t6):.3f}", flush=True)
