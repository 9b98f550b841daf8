"""Child program of tests/test_gpu_dist_backend.py: BayesianOptimization over the REAL device backend
(DeviceBackend: sharded fused predict, top-q record exchange, HVI select, gathered state arrays,
rank-0 objective) with every rank of a torch.distributed group on the one GPU of the box.

    python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 --master-port PORT \
        tests/helpers/dist_orchestrator_run.py OUT_PREFIX [gloo]

With P = 1 (or no torch.distributed.run) it runs the single-rank loop.  Each rank writes
OUT_PREFIX.rank<r>.json: per case the trajectory (x, y), the fitted hyper-parameters, the returned
count, how often the objective ran on this rank and what its callbacks saw."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CASES = [("sum_ucb", 3), ("hvi", 3), ("sum_ucb", 50)]


def main():
    out = sys.argv[1]
    backend = sys.argv[2] if len(sys.argv) > 2 else "gloo"
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group(backend)
    rank = dist.get_rank() if world > 1 else 0
    torch.cuda.set_device(0)
    import bayesopt_smart_amd as bo
    res = {}
    for acq, batch in CASES:
        calls = [0]
        seen = []

        def toy(p):
            calls[0] += 1
            p = np.asarray(p, dtype=np.float64)
            return np.array([-((p[0] - 30) ** 2) + 100.0, -((p[1] - 20) ** 2) + 20.0])

        np.random.seed(42)
        cb = [lambda st: seen.append(float(np.asarray(st["acquisition_values"]).sum()))] if rank == 0 else None
        opt = bo.BayesianOptimization(toy, [(0, 64), (0, 48)], n_objectives=2, initial_samples=6, n_iterations=3,
                                      batch_size=batch, betas=np.array([2.0, 2.0]), acquisition=acq,
                                      reference_point=np.array([-5000.0, -3000.0]), device="cuda:0", callbacks=cb)
        opt.optimize()
        res[f"{acq}-{batch}"] = {"x": opt.x_vector.tolist(), "y": opt.y_vector.tolist(),
                                 "ls": opt.length_scales.tolist(), "pv": opt.prior_variance.tolist(),
                                 "n": int(opt.n_evaluations), "calls": calls[0], "seen": seen}
    with open(f"{out}.rank{rank}.json", "w") as fh:
        json.dump(res, fh)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
