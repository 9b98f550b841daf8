"""Where one single-objective compute_mll call's time goes (the Powell fit's call pattern: one
objective, a new length scale per call), for rocprofv3 --kernel-trace.

    python scripts/mll_call_probe.py [cfg=C3] [calls=200]          (GPU: wall time per call)
    python scripts/mll_call_probe.py trace=<kernel_trace.csv>      (CPU: the trace's timeline)

The timeline splits each call into: the init kernel, the gap init -> persistent kernel, the
persistent kernel, and the gap to the next call's init (host completion wait + the next launch)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
args = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)

if "trace" in args:
    import csv
    rows = list(csv.DictReader(open(args["trace"])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
                if "fit_" in r["Kernel_Name"])
    calls, cur = [], None
    for s, e, name in ev:
        if "fit_init_kernel" in name:
            cur = [s, e]
            calls.append(cur)
        elif cur is not None and len(cur) == 2:
            cur += [s, e]
    calls = [c for c in calls if len(c) == 4][5:]          # steady state
    init = np.array([c[1] - c[0] for c in calls]) / 1e3
    gap1 = np.array([c[2] - c[1] for c in calls]) / 1e3
    pers = np.array([c[3] - c[2] for c in calls]) / 1e3
    gap2 = np.array([b[0] - a[3] for a, b in zip(calls, calls[1:])]) / 1e3
    per = np.array([b[0] - a[0] for a, b in zip(calls, calls[1:])]) / 1e3
    med = lambda v: f"{np.median(v):7.2f}"  # noqa: E731
    print(f"{len(calls)} calls (us, medians): init {med(init)} | gap {med(gap1)} | persistent {med(pers)} | "
          f"to next call {med(gap2)} | call period {med(per)}")
    sys.exit(0)

import torch  # noqa: E402
import bayesopt_smart_amd as bo  # noqa: E402
import bench  # noqa: E402
from bayesopt_smart_amd import kernels as K  # noqa: E402

cfg = bench.CONFIGS[args.get("cfg", "C3")]
calls = int(args.get("calls", 200))
x, y, pm, pv, ls, betas, _, _ = bench.make_config_problem(cfg, 1)
n, n_obj = x.shape[0], len(pm)
dev = torch.device("cuda", 0)
xd, yd = torch.tensor(x, device=dev), torch.tensor(y, device=dev)
km = torch.zeros((n_obj, n, n), dtype=torch.float64, device=dev)
rng = np.random.default_rng(0)
ts = []
for i in range(calls):
    lsv = np.array(ls, dtype=np.float64) * rng.uniform(0.7, 1.3, size=n_obj)
    t0 = time.perf_counter()
    K._mll_terms(xd, yd, km, pm, pv, lsv, n, [0])
    ts.append(time.perf_counter() - t0)
ts = np.array(ts[10:]) * 1e6
print(f"{args.get('cfg', 'C3')} N={n}: single-objective compute_mll wall per call: median {np.median(ts):.1f} us, "
      f"p10 {np.percentile(ts, 10):.1f}, p90 {np.percentile(ts, 90):.1f}", flush=True)
