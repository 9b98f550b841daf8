"""Standalone selection micro-benchmark: bo_select_topq (select_next_batch over a stored
acquisition array, acquisition.py:116-144) per call, HIP-graph replayed (no host launch cost in
the figure), with the evaluated points excluded; checked against numpy's order.

    python scripts/select_ubench.py [--cases C3,C5] [--reps 50]

One JSON line per case and exclusion form (points: the per-call hash set, bo_select_topq;
masked: the persistent exclusion mask, bo_select_topq_masked): us per call (selection kernel + final merge), GB/s on the 8 B per
candidate read, fraction of 8 TB/s.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesopt_smart_amd as bo  # noqa: E402
from bayesopt_smart_amd import _lib  # noqa: E402

CASES = {  # name: (grid side0, side1, n evaluated, q)
    "C2": (512, 512, 128, 3),
    "C3": (1024, 1024, 512, 3),
    "C3q16": (1024, 1024, 512, 16),
    "C3q48": (1024, 1024, 512, 48),
    "C3noex": (1024, 1024, 0, 3),
    "C3q1": (1024, 1024, 512, 1),
    "C3q1noex": (1024, 1024, 0, 1),
    "C3q16noex": (1024, 1024, 0, 16),
    "C5": (2048, 2048, 2048, 16),
}


def run(name, reps, masked=False):
    s0, s1, n_ev, q = CASES[name]
    m = s0 * s1
    rng = np.random.default_rng(1)
    acq_h = rng.standard_normal(m)
    lin = rng.choice(m, n_ev, replace=False)
    ev = np.stack([lin // s1, lin % s1], axis=1).astype(np.float64)
    acq_h[lin[: n_ev // 4]] += 10.0                          # some evaluated points at the top
    dev = torch.device("cuda:0")
    acq = torch.tensor(acq_h, device=dev)
    xd = torch.tensor(ev, device=dev) if n_ev else torch.zeros((1, 2), dtype=torch.float64, device=dev)
    lib = _lib.load()
    ws = torch.empty(lib.bo_select_topq_workspace_size(m, q), dtype=torch.uint8, device=dev)
    tv = torch.empty(q, dtype=torch.float64, device=dev)
    ti = torch.empty(q, dtype=torch.int64, device=dev)
    glo = (ctypes.c_int64 * 8)(*([0] * 8))
    gsh = (ctypes.c_int64 * 8)(*([s0, s1] + [1] * 6))

    cands = bo.predict.CandidateSet.grid([(0, s0), (0, s1)])
    mask = bo.acquisition.ExclusionMask(cands, 0, m, dev).update(ev)

    def call():
        if masked:
            _lib.check(lib.bo_select_topq_masked(acq.data_ptr(), m, 0, mask.ptr, q, tv.data_ptr(), ti.data_ptr(),
                                                 ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream),
                       "select_masked")
            return
        _lib.check(lib.bo_select_topq(acq.data_ptr(), m, cands.kind_code,
                                      None, glo, gsh, 2, 0, xd.data_ptr(), n_ev, q, tv.data_ptr(),
                                      ti.data_ptr(), ws.data_ptr(), ws.numel(),
                                      torch.cuda.current_stream().cuda_stream), "select")
    call()
    torch.cuda.synchronize()
    excl = np.zeros(m, dtype=bool)
    excl[lin] = True
    want = np.lexsort((np.arange(m), -np.where(excl, -np.inf, acq_h)))[:q]
    ok = bool(np.array_equal(ti.cpu().numpy(), want))
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            call()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            call()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(json.dumps({"case": name, "masked": masked, "n_cand": m, "n_excl": n_ev, "q": q, "us_per_call": round(us, 2),
                      "GBps": round(8 * m / (us * 1e-6) / 1e9, 1),
                      "hbm_frac": round(8 * m / (us * 1e-6) / 1e9 / 8000.0, 4), "matches_numpy": ok}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    for c in args.cases.split(","):
        for masked in (False, True):
            run(c, args.reps, masked)


if __name__ == "__main__":
    main()
