"""Child of tests/test_gpu_rccl_one_rank.py, launched by torch.distributed.run with one rank:
the drop-in loop (BayesianOptimization.optimize through DeviceBackend, with a callback so the
state arrays are gathered) and the hypervolume accumulator, first with the RCCL process group and
BO_FORCE_COLLECTIVES=1 (every collective of the loop runs: the top-q all_gather, the callbacks
flag all_reduce, the y broadcast, the state gathers, the front-HV all_reduce), then again after
destroy_process_group (no collectives); prints both trajectories."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, sys.argv[1])
os.environ["BO_FORCE_COLLECTIVES"] = "1"
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)

from bayesopt_smart_amd.bayesian_optimization import BayesianOptimization  # noqa: E402
from bayesopt_smart_amd.distributed import collectives_on, front_hypervolume  # noqa: E402
from bayesopt_smart_amd.pareto import is_pareto_efficient  # noqa: E402


def toy(x):
    return np.array([-((x[0] - 150) ** 2) + 100, -((x[1] - 150) ** 2) + 20], dtype=np.float64)


def run():
    seen = []
    np.random.seed(42)
    opt = BayesianOptimization(toy, [(0, 300), (0, 300)], n_objectives=2, initial_samples=6, n_iterations=3,
                               batch_size=3, betas=np.array([2.0, 2.0]), device=dev,
                               callbacks=[lambda s: seen.append(float(np.asarray(s["acquisition_values"]).sum()))])
    opt.optimize()
    y = opt.y_vector[: opt.n_evaluations]
    front = y[is_pareto_efficient(y)]
    hv = front_hypervolume(front, y.min(0) - 1.0, device=dev)
    return dict(x=opt.x_vector.tolist(), acq_sums=seen, hv=hv)


res = {"backend": dist.get_backend(), "collectives": collectives_on()}
res["rccl"] = run()
dist.destroy_process_group()
res["collectives_after"] = collectives_on()
res["plain"] = run()
print("RESULT " + json.dumps(res))
