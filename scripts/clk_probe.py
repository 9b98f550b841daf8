"""The core clock the fused C3 kernel runs at, from inside the kernel (diagnostic build
BO_BUILD_VARIANT=DEF_PREDICT_CLK: every wave of cm_tiles records its shader-clock (s_memtime) and
100 MHz real-time-clock (s_memrealtime) spans; bo_debug_predict_clk reads them back).

    BO_AMD_LIB=.../libbo_amd_def_predict_clk.so python scripts/clk_probe.py [cfg=C3] [reps=5]

Prints, per launch: the event-timed kernel ms, the mean core clock over the waves
(sum clock / sum realtime x 100 MHz), the spread of the waves' spans, and the MFMA-bound time at
that clock (executed MFMAs per SIMD x 64 cycles / clock) -- so the kernel's distance from its
roof splits into "clock below 2.4 GHz" and "cycles not issuing MFMAs"."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo  # noqa: E402
import bench  # noqa: E402

args = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)
cfg_name = args.get("cfg", "C3")
reps = int(args.get("reps", 5))
idle_ms = float(args.get("idle_ms", 0))          # host idle before each timed launch (DVFS ramp)
cfg = bench.CONFIGS[cfg_name]
x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(cfg, 1)
c = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])]) if cand[0] == "grid" else cand[1]
dev = torch.device("cuda", 0)
xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
L = bo._lib.load()
L.bo_debug_predict_clk.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.bo_debug_predict_clk.restype = ctypes.c_int
call = bo.predict_acquire(xd, yd, kd, c, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=cfg["q"],
                          device=dev, prepare=True)
n = x.shape[0]
m = cand[1] * cand[2] if cand[0] == "grid" else c.n
mfma_flops = bench.executed_mfma_flops_per_candidate("upper", n, len(pm)) * m
mfma_per_simd = mfma_flops / 2048 / 1024                    # 256 CUs x 4 SIMDs
import time  # noqa: E402
for r in range(reps + 2):
    call()
    torch.cuda.synchronize()
    if idle_ms > 0:
        time.sleep(idle_ms / 1000.0)
    L.bo_profile_start(1)
    call()
    torch.cuda.synchronize()
    ms, k = ctypes.c_double(), ctypes.c_int()
    L.bo_profile_stop(ctypes.byref(ms), ctypes.byref(k))
    buf = np.zeros(2 * 4096, dtype=np.int64)
    nw = L.bo_debug_predict_clk(buf.ctypes.data, 4096)
    spans = buf[: 2 * nw].reshape(-1, 2)
    spans = spans[spans[:, 1] > 0]
    if r < 2:
        continue
    f_ghz = spans[:, 0].sum() / spans[:, 1].sum() * 0.1
    rt_ms = spans[:, 1] / 1e5
    mfma_ms = mfma_per_simd * 64 / (f_ghz * 1e9) * 1e3
    print(f"{cfg_name} (idle {idle_ms:g} ms before): kernel {ms.value:.3f} ms; waves {len(spans)}; core clock {f_ghz:.3f} GHz "
          f"(per-wave min {spans[:, 0].min() / spans[:, 1].max() * 0.1:.3f}); wave span {rt_ms.min():.3f} .. "
          f"{rt_ms.max():.3f} ms; MFMA-bound time at that clock {mfma_ms:.3f} ms "
          f"({mfma_ms / ms.value:.3f} of the kernel), at 2.4 GHz {mfma_per_simd * 64 / 2.4e9 * 1e3:.3f} ms",
          flush=True)
