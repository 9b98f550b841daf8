"""The RCCL (torch.distributed "nccl") exchange path on ONE GPU: torch.distributed.run with one
rank and BO_FORCE_COLLECTIVES=1, so that every collective the multi-GPU run uses executes over
RCCL -- bench.py's step (the device-tensor all_gather_into_tensor of the top-q records, the
max-over-ranks all_reduce, the barriers), the drop-in loop's --iteration mode, and the loop
itself through BayesianOptimization (tests/helpers/rccl_loop.py: the exchange, the callbacks flag
all_reduce, the y broadcast, the state gathers, the hypervolume accumulator).  Results must equal
the same runs without a process group (bayesian_optimization.py:108-247's trajectory, the
bench's selected batch).  The 8-GPU run itself is the driver's."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, dist_launch, timeout=300):
    env = dict(os.environ, BO_FORCE_COLLECTIVES="1" if dist_launch else "0")
    cmd = [sys.executable]
    if dist_launch:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
                "127.0.0.1", "--master-port", str(_port())]
    r = subprocess.run(cmd + args, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    return r.stdout


def _json_line(out):
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def test_bench_step_over_rccl_one_rank():
    args = ["bench.py", "--gpus", "1", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    got = _json_line(_run(args, True))
    ref = _json_line(_run(args, False))
    assert got["collectives"]["backend"] == "nccl" and got["collectives"]["world_size"] == 1, got.get("collectives")
    assert "collectives" not in ref
    assert got["selected"] == ref["selected"]
    assert got["select_standalone"]["matches_fused_selection"] is True


def test_bench_iteration_over_rccl_one_rank():
    args = ["bench.py", "--iteration", "--config", "C3", "--steps", "1", "--warmup", "1"]
    got = _json_line(_run(args, True))
    ref = _json_line(_run(args, False))
    assert [r["n_train"] for r in got["per_iteration_ms"]] == [r["n_train"] for r in ref["per_iteration_ms"]]
    assert got["fitted_length_scales"] == ref["fitted_length_scales"]


def test_drop_in_loop_over_rccl_one_rank():
    out = _run([os.path.join("tests", "helpers", "rccl_loop.py"), ROOT], True)
    res = json.loads(next(ln for ln in out.splitlines() if ln.startswith("RESULT "))[7:])
    assert res["backend"] == "nccl" and res["collectives"] is True and res["collectives_after"] is False
    assert res["rccl"]["x"] == res["plain"]["x"]
    assert res["rccl"]["acq_sums"] == res["plain"]["acq_sums"]
    assert res["rccl"]["hv"] == res["plain"]["hv"]
