"""Benchmark of the north-star hot path: GP predict + acquisition (Sigma-UCB "HVI") + top-q.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2], "C3"): 2-D / 2-objective toy_function
(examples/benchmark_functions.py:33-50), N_train = 512, 1,048,576 candidates per GPU on the
reference's integer 'ij' grid (bayesian_optimization.py:338-340), length scales 20, betas 2,
q = 3 (select_next_batch with the evaluated points excluded).  Weak scaling: rank r scores
rows [1024 r, 1024 (r + 1)) of a (1024 N) x 1024 grid; the per-rank top-q lists meet in one
RCCL all_gather, merged on rank 0.

One step = one bo_predict_acquire call per rank (K^-1 packing, alpha = K^-1 (y - pm), the
fused predict/acquisition kernel writing mu, var and acq for every candidate, the top-q
merge) + the global top-q exchange + the indices on the host.  Inputs (X, y, K^-1) are
resident in HBM before the timed region.

Prints ONE JSON line (rank 0).  `roofline` is the fused kernel's f64 matrix-core throughput
(algorithmic flops F per candidate) over its HIP-event-timed launches;
`cpu_baseline` times the C/OpenMP restatement of the reference algorithm (oracle/cpu_ref.c)
on a bounded slice of the same workload on this host's cores.
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_TRAIN = 512
SIDE = 1024
N_OBJ = 2
DIM = 2
TOPQ = 3
LS = 20.0
BETA = 2.0
PEAK_F64_MATRIX_TFLOPS = 78.6        # MI355X dense FP64 matrix peak (datasheet)
PEAK_HBM_GBPS = 8000.0


def flops_per_candidate(n=N_TRAIN, n_obj=N_OBJ, d=DIM):
    """F = nobj (2N^2 + 6N) + (3d - 1) N (reference formulation)."""
    return n_obj * (2 * n * n + 6 * n) + (3 * d - 1) * n


def executed_mfma_flops_per_candidate(mode, n=N_TRAIN, n_obj=N_OBJ):
    """Matrix-core flops the fused kernel actually issues per candidate (16x16x4 f64 MFMA,
    2048 flops, 16 candidates per wave): dense walks all (NS/8) E-pairs x (NS/2) k-step pairs,
    upper only the blocks ep <= c (q = 2 k.(U k), U = upper triangle of sym(K^-1))."""
    ns = -(-n // 4)
    ns = next(v for v in (8, 16, 32, 64, 96, 128) if v >= ns) if n <= 512 else ns
    pairs = ns * ns // 16 if mode == "dense" else ns * ns // 32 + ns // 4
    return n_obj * pairs * 4 * 2048 // 16


def toy_function(x):
    """examples/benchmark_functions.py:33-50."""
    return np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20], axis=1)


def make_problem(world):
    rng = np.random.default_rng(0)
    rows = SIDE * world
    lin = rng.choice(rows * SIDE, size=N_TRAIN, replace=False)
    x = np.stack([lin // SIDE, lin % SIDE], axis=1).astype(np.float64)
    y = toy_function(x)
    pm, pv = y.mean(0), y.var(0)                               # compute_prior_mean / _variance
    ls = np.full(N_OBJ, LS)
    betas = np.full(N_OBJ, BETA)
    # K + 1e-6 I and its inverse (update_k / invert_k, numba_kernels.py:329-403): setup only
    diff = x[:, None, :] - x[None, :, :]
    sq = np.einsum("ijd,ijd->ij", diff, diff)
    kinv = np.stack([np.linalg.inv(pv[o] * np.exp(-0.5 * sq / ls[o] ** 2) + 1e-6 * np.eye(N_TRAIN))
                     for o in range(N_OBJ)])
    return x, y, pm, pv, ls, betas, kinv, rows


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(x, y, pm, pv, ls, betas, kinv, budget_s=12.0, chunk=16384, max_cand=SIDE * SIDE):
    """Reference algorithm on the host cores: oracle/cpu_ref.c, the C/OpenMP restatement of
    update_k_star -> update_mean -> update_variance (materialised K* per candidate block,
    DGEMM K^-1 K*, the serial quadratic form) -> standardise -> UCB -> Sigma-UCB, then
    select_next_batch's full descending sort + exclusion walk."""
    from oracle import cpu_ref
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cpu_ref.load()
    done = 0
    acqs = []
    t0 = time.perf_counter()
    while done < max_cand and time.perf_counter() - t0 < budget_s:
        lin = np.arange(done, done + chunk)
        pts = np.stack([lin // SIDE, lin % SIDE], axis=1).astype(np.float64)
        acqs.append(cpu_ref.predict_acquire(x, y, pts, kinv, pm, pv, ls, betas, threads=threads,
                                            outputs=True)["acq"])
        done += chunk
    lin = np.arange(done)
    cpu_ref.select(np.concatenate(acqs), np.stack([lin // SIDE, lin % SIDE], axis=1).astype(np.float64),
                   x, TOPQ)
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "candidate-points/sec", "cores": threads, "kind": "port",
            "sample": f"first {done} candidates of the C3 grid (N_train=512, 2 objectives, mu/var/acq "
                      f"written, top-{TOPQ} select), oracle/cpu_ref.c (C/OpenMP, {threads} threads of "
                      f"{os.cpu_count()} logical CPUs, {_cpu_model()}), {dt:.1f} s"}


def pmc_traffic():
    """HBM bytes per fused-kernel launch from the committed rocprofv3 PMC summary, if any."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
            if d.get("workload") == "C3" and d.get("hbm_bytes_per_launch"):
                return float(d["hbm_bytes_per_launch"])
        except Exception:
            pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=("auto", "dense"), default="auto",
                    help="variance formulation (auto = 2 k.(U k) with U = triu(sym(K^-1)), diagonal halved)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import bayesopt_smart_amd as bo
    lib = bo._lib.load()

    x, y, pm, pv, ls, betas, kinv, rows = make_problem(world)
    cands = bo.CandidateSet.grid([(0, rows), (0, SIDE)])
    per_rank = SIDE * SIDE
    offset = rank * per_rank
    xd = torch.tensor(x, device=dev)
    yd = torch.tensor(y, device=dev)
    kd = torch.tensor(kinv, device=dev)
    out = {"mu": torch.empty((N_OBJ, per_rank), dtype=torch.float64, device=dev),
           "var": torch.empty((N_OBJ, per_rank), dtype=torch.float64, device=dev),
           "acq": torch.empty(per_rank, dtype=torch.float64, device=dev)}
    gath_v = torch.empty(world * TOPQ, dtype=torch.float64, device=dev)
    gath_i = torch.empty(world * TOPQ, dtype=torch.int64, device=dev)

    def step():
        r = bo.predict_acquire(xd, yd, kd, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"),
                               topq=TOPQ, offset=offset, count=per_rank, out=out, device=dev,
                               mode=args.mode)
        if world > 1:
            dist.all_gather_into_tensor(gath_v, r["top_val"])
            dist.all_gather_into_tensor(gath_i, r["top_idx"])
            v, i = gath_v.cpu().numpy(), gath_i.cpu().numpy()
        else:
            v, i = r["top_val"].cpu().numpy(), r["top_idx"].cpu().numpy()
        return bo.merge_topq(v, i, TOPQ)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    lib.bo_profile_start(args.steps)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sel = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    import ctypes
    kms, nl = ctypes.c_double(), ctypes.c_int()
    lib.bo_profile_stop(ctypes.byref(kms), ctypes.byref(nl))
    t_step = dt / args.steps
    if world > 1:
        tt = torch.tensor([t_step, kms.value / max(nl.value, 1)], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_step, k_ms = tt.tolist()
    else:
        k_ms = kms.value / max(nl.value, 1)

    if rank == 0:
        f = flops_per_candidate()
        fx = executed_mfma_flops_per_candidate(args.mode)
        achieved = f * per_rank / (k_ms * 1e-3) / 1e12
        res = {
            "metric": "candidate-points/sec (GP predict + HVI) at N_train=512, N_cand=1M",
            "value": world * per_rank / t_step,
            "unit": "candidate-points/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_step * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (toy_function on a seeded 512-point design)",
            "config": {"workload": "C3: 2D/2-obj toy_function, N_train=512, N_cand=1,048,576 per GPU "
                                   "('ij' integer grid), HVI (Sigma-UCB), q=3",
                       "n_train": N_TRAIN, "n_cand_per_gpu": per_rank, "n_objectives": N_OBJ,
                       "dim": DIM, "topq": TOPQ, "parallelism": f"candidate-shard x{world}"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_F64_MATRIX_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / PEAK_F64_MATRIX_TFLOPS,
                         "traffic": pmc_traffic(),
                         "kernel": ("cm_predict_kernel<2, true, true>" if args.mode == "auto"
                                    else "cm_predict_kernel<2, true, false>"),
                         "kernel_ms": k_ms, "flops_per_candidate": f,
                         "formulation": ("upper: q = 2 k.(U k), U = triu((K^-1 + K^-T)/2), diag/2" if args.mode == "auto"
                                         else "dense: q = k^T (K^-1 k)"),
                         "executed_mfma_flops_per_candidate": fx,
                         "executed_mfma_tflops": fx * per_rank / (k_ms * 1e-3) / 1e12,
                         "executed_mfma_frac": fx * per_rank / (k_ms * 1e-3) / 1e12 / PEAK_F64_MATRIX_TFLOPS},
            "selected": [int(i) for i in sel[1]],
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(x, y, pm, pv, ls, betas, kinv)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
