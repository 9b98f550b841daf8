"""The multi-rank loop over the REAL device backend: BayesianOptimization with
sum_ucb, the exact HVI and a batch above BO_MAX_TOPQ (the gathered-array selection), P = 2 ranks of
a gloo group sharing the box's GPU (the RCCL transport is the only part not exercised), against the
single-rank run: identical trajectory (x, y), fitted hyper-parameters and returned count; the
objective runs on rank 0 only (the initial design included); a callback registered on rank 0 alone
sees the gathered acquisition array of the single-rank run (the collective gather is decided
collectively, so the other rank's collectives stay matched)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SCRIPT = os.path.join(HERE, "helpers", "dist_orchestrator_run.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(world, out):
    env = dict(os.environ, PYTHONPATH=ROOT)
    if world == 1:
        cmd = [sys.executable, SCRIPT, out]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), SCRIPT, out, "gloo"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return [json.load(open(f"{out}.rank{k}.json")) for k in range(world)]


def test_two_ranks_match_one_rank(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    one = _run(1, str(tmp_path / "w1"))[0]
    two = _run(2, str(tmp_path / "w2"))
    for case, ref in one.items():
        for r, got in enumerate(two):
            g = got[case]
            assert g["x"] == ref["x"], (case, r)
            assert g["y"] == ref["y"], (case, r)
            assert g["ls"] == ref["ls"] and g["pv"] == ref["pv"], (case, r)
            assert g["n"] == ref["n"]
        assert two[0][case]["calls"] == ref["calls"] > 0, case       # every evaluation on rank 0 ...
        assert two[1][case]["calls"] == 0, case                      # ... and none on rank 1
        np.testing.assert_allclose(two[0][case]["seen"], ref["seen"], rtol=1e-12)
        assert two[1][case]["seen"] == []
