import os, sys, json, ctypes, subprocess
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
code = r'''
import os, sys, json, ctypes, numpy as np, torch
sys.path.insert(0, os.getcwd())
os.environ["BO_AMD_LIB"] = sys.argv[1]
import bench, bayesopt_smart_amd as bo
cfg = bench.CONFIGS[sys.argv[3]]
x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(cfg, 1)
c = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])]) if cand[0] == "grid" else bo.CandidateSet.explicit(cand[1][: 1 << 20], device="cuda")
xd, yd, kd = (torch.tensor(a, device="cuda") for a in (x, y, kinv))
L = bo._lib.load()
go = lambda: bo.predict_acquire(xd, yd, kd, c, pm, pv, ls, betas, outputs=("acq",), topq=3, mode=sys.argv[2])
go(); torch.cuda.synchronize()
ts = []
for _ in range(3):
    L.bo_profile_start(1); go(); torch.cuda.synchronize()
    ms, n = ctypes.c_double(), ctypes.c_int(); L.bo_profile_stop(ctypes.byref(ms), ctypes.byref(n)); ts.append(ms.value)
print(json.dumps({"lib": os.path.basename(sys.argv[1]), "mode": sys.argv[2], "cfg": sys.argv[3], "median_ms": float(np.median(ts))}))
'''
for rnd in range(2):
    for lib in sys.argv[1:]:
        for mode, cfgname in [tuple(a.split(":")) for a in os.environ.get("AB_CASES", "auto:C3,auto:C4,fp32:C5").split(",")]:
            r = subprocess.run([sys.executable, "-c", code, lib, mode, cfgname], capture_output=True, text=True)
            print(r.stdout.strip() or r.stderr[-1500:], flush=True)
