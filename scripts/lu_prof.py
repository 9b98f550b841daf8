"""invert_k's LU fallback timing: C3's design at a fitted-like length scale (Cholesky fails,
numba_kernels.py:370-403 falls back to np.linalg.inv) -- wall vs HIP events, for rocprofv3."""
import sys, time
import numpy as np
import torch
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo
import bench

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"]
ls_fit = float(sys.argv[2]) if len(sys.argv) > 2 else 680.0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
x, y, pm, pv, ls, betas, _, _ = bench.make_config_problem(cfg, 1)
if len(sys.argv) > 4 and int(sys.argv[4]) > x.shape[0]:       # N above the config's: extra grid points
    extra = np.random.default_rng(5).choice(1024 * 1024, size=int(sys.argv[4]) - x.shape[0], replace=False)
    xe = np.stack([extra // 1024, extra % 1024], 1).astype(np.float64)
    x = np.concatenate([x, xe if x.shape[1] == 2 else np.resize(xe, (xe.shape[0], x.shape[1]))])
n, n_obj = x.shape[0], len(pm)
dev = torch.device("cuda", 0)
xd = torch.tensor(x, device=dev)
km = torch.zeros((n_obj, n, n), dtype=torch.float64, device=dev)
bo.kernels.update_k(km, xd, 0, n, pv, np.full(n_obj, ls_fit))
g = lambda: bo.kernels.invert_k(n, km, lu_hint=[True] * n_obj)   # straight to the LU path
before = bo._lib.fit_path_counts()
g(); torch.cuda.synchronize()
print("fit paths after one call:", {k: v - before.get(k, 0) for k, v in bo._lib.fit_path_counts().items()})
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
e0.record()
for _ in range(reps):
    t0 = time.perf_counter(); g(); ts.append(time.perf_counter() - t0)
e1.record(); torch.cuda.synchronize()
print(f"invert_k (LU fallback) N={n} ls={ls_fit}: wall median {np.median(ts)*1e3:.3f} ms, "
      f"events {e0.elapsed_time(e1)/reps:.3f} ms per call", flush=True)

# diagnostic build: the LU phase stamps of one more call (step launches: 1 start, 2 pending step
# applied, 3 strip factored, 4 permutation record written; solve workgroup 0: 8 forward step,
# 9 permutation applied, 12 backward step)
lib = bo._lib.load()
if hasattr(lib, "bo_debug_lu_timing"):
    import ctypes
    buf = (ctypes.c_longlong * 8192)()
    lib.bo_debug_lu_timing(buf, 4096)
    g(); torch.cuda.synchronize()
    cnt = lib.bo_debug_lu_timing(buf, 4096)
    ev = sorted((buf[2 * i + 1], buf[2 * i] >> 16, (buf[2 * i] >> 4) & 4095, buf[2 * i] & 15) for i in range(cnt))
    t0 = ev[0][0]
    rows = {}
    for t, k, slot, tag in ev:
        rows.setdefault((tag >= 8, k, slot), {})[tag] = (t - t0) * 0.01
    for key in sorted(rows, key=lambda q: min(rows[q].values())):
        print("solve" if key[0] else "step", key[1], "slot", key[2],
              " ".join(f"{tag}:{v:.2f}" for tag, v in sorted(rows[key].items())))
if hasattr(lib, "bo_debug_lu_cols"):
    import ctypes
    cb = (ctypes.c_longlong * 4096)()
    lib.bo_debug_lu_cols(cb, 4096)
    for k in (0, 1, 2):
        print(f"panel step {k}: per column [max found, after barrier, updated] - start (us), then to next column")
        for j in range(16):
            b0 = (k * 16 + j) * 4
            nxt = cb[b0 + 4] if j < 15 else cb[b0 + 3]
            print("  col", j, " ".join(f"{(cb[b0 + t] - cb[b0]) * 0.01:.2f}" for t in (1, 2, 3)), f"{(nxt - cb[b0]) * 0.01:.2f}")
if hasattr(lib, "bo_debug_lu_cclk"):
    import ctypes
    cw = (ctypes.c_longlong * 4096)()
    cc = (ctypes.c_longlong * 4096)()
    lib.bo_debug_lu_cols(cw, 4096)
    lib.bo_debug_lu_cclk(cc, 4096)
    for k in (0, 1, 2, 16, 30):
        b0, b1 = (k * 16) * 4, (k * 16 + 15) * 4 + 3
        dw, dc = (cw[b1] - cw[b0]) * 10e-9, cc[b1] - cc[b0]
        if dw > 0:
            print(f"panel step {k}: {dw*1e6:.2f} us wall, {dc} shader clocks -> {dc/dw/1e9:.3f} GHz; "
                  f"per column {dc/16:.0f} clocks [" + " ".join(
                      f"{cc[(k*16+j)*4+t]-cc[(k*16+j)*4+t-1]}" for j in (0, 8) for t in (1, 2, 3)) + "]")
