"""Where the drop-in loop's 'acquisition' time goes at C3: DeviceBackend.select timed with a
synchronisation before it (work still in flight from the fit), and predict_acquire alone on the
same inputs right after."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench
import bayesopt_smart_amd as bo
from bayesopt_smart_amd.bayesian_optimization import optimize, DeviceBackend

cfg = bench.CONFIGS["C3"]
x, y, pm, pv, ls, betas, _, cand = bench.make_config_problem(cfg, 1)
n, q = cfg["n_train"], cfg["q"]
cands = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])])
total = n + 4 * q
dev = torch.device("cuda", 0)


class Probe(DeviceBackend):
    def select(self, fitted, *a, **k):
        t0 = time.perf_counter(); torch.cuda.synchronize(); t1 = time.perf_counter()
        r = super().select(fitted, *a, **k)
        torch.cuda.synchronize(); t2 = time.perf_counter()
        xd, yd, kinv = fitted
        print(f"  select: pending before {1e3 * (t1 - t0):.3f} ms, select {1e3 * (t2 - t1):.3f} ms; "
              f"kinv {tuple(kinv.shape)} stride {kinv.stride()} xd {tuple(xd.shape)} yd {tuple(yd.shape)} "
              f"dtype {kinv.dtype}", flush=True)
        out = self._outputs()
        t3 = time.perf_counter()
        bo.predict_acquire(xd, yd, kinv, self.cands, a[0], a[1], a[2], a[3], outputs=tuple(out), topq=q, out=out,
                           device=self.dev)
        torch.cuda.synchronize()
        print(f"  predict_acquire alone {1e3 * (time.perf_counter() - t3):.3f} ms", flush=True)
        return r


xv = np.zeros((total, 2)); yv = np.zeros((total, 2)); xv[:n] = x; yv[:n] = y
be = Probe(cands, 2, total, dev)
optimize(xv, yv, None, None, None, None, None, None, None, None, cands, pm, pv.copy(), None, n, total, 2,
         lambda p: bench.toy_function(np.asarray(p, dtype=np.float64)[None])[0], betas, ls.copy(), q, None,
         backend=be)
