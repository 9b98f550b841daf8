"""sha256 of one fused call's outputs (mu, var, acq, top-q) for a bench config, with the library
named by BO_AMD_LIB: two builds that must be bit-identical (a code-placement change, a peel) are
checked by comparing the printed digests.

    BO_AMD_LIB=.../lib.so python scripts/lib_outputs_sha.py C3 [mode]"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo  # noqa: E402
import bench  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C3"
mode = sys.argv[2] if len(sys.argv) > 2 else ("fp32" if cfg_name == "C5" else "auto")
cfg = bench.CONFIGS[cfg_name]
x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(cfg, 1)
c = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])]) if cand[0] == "grid" else cand[1]
n = cand[1] * cand[2] if cand[0] == "grid" else min(c.n, 1 << 20)
r = bo.predict_acquire(x, y, kinv, c, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=cfg["q"], count=n,
                       mode=mode)
torch.cuda.synchronize()
h = hashlib.sha256()
for k in ("mu", "var", "acq", "top_val", "top_idx"):
    h.update(r[k].cpu().numpy().tobytes())
print(f"{cfg_name} {mode} {os.path.basename(os.environ.get('BO_AMD_LIB', 'libbo_amd.so'))}: {h.hexdigest()[:24]}",
      flush=True)
