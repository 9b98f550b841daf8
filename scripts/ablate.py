"""Time the fused kernel of a bench config in several library builds (ablation / A-B),
interleaved in one process per library (§5.4 rule 24 of the CDNA guide: compare within one
device session).

    python scripts/ablate.py lib1.so lib2.so ... [mode=auto] [cfg=C3]   (one line per lib)
"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def run_one(lib, mode, rounds, cfg="C3"):
    code = f"""
import os, sys, json, ctypes, numpy as np, torch
sys.path.insert(0, {ROOT!r})
os.environ['BO_AMD_LIB'] = {lib!r}
import bench, bayesopt_smart_amd as bo
C = bench.CONFIGS[{cfg!r}]
x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(C, 1)
c = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])]) if cand[0] == 'grid' else cand[1]
xd, yd, kd = (torch.tensor(a, device='cuda') for a in (x, y, kinv))
L = bo._lib.load()
def go():
    return bo.predict_acquire(xd, yd, kd, c, pm, pv, ls, betas, outputs=('mu', 'var', 'acq'), topq=C['q'], mode={mode!r})
for _ in range(3): go()
torch.cuda.synchronize()
ts = []
for _ in range({rounds}):
    L.bo_profile_start(1); go(); torch.cuda.synchronize()
    ms, n = ctypes.c_double(), ctypes.c_int(); L.bo_profile_stop(ctypes.byref(ms), ctypes.byref(n))
    ts.append(ms.value)
print(json.dumps({{'lib': os.path.basename({lib!r}), 'cfg': {cfg!r}, 'mode': {mode!r}, 'median_ms': float(np.median(ts)), 'min_ms': float(np.min(ts))}}))
"""
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)


if __name__ == "__main__":
    libs = [os.path.abspath(a) for a in sys.argv[1:] if a.endswith(".so")]   # dlopen needs a path
    modes = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("mode=")] or ["auto"]
    cfgs = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("cfg=")] or ["C3"]
    for rnd in range(2):
        for cfg in cfgs:
            for lib in libs:
                for mode in modes:
                    r = run_one(lib, mode, 7, cfg)
                    print(r.stdout.strip() or r.stderr[-2000:], flush=True)
