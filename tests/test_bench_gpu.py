"""bench.py's multi-rank path, rehearsed on one GPU: the launcher
the driver's N-GPU runs use (`--gpus N` starting N rank processes with the torchrun
environment), the process group, the barrier-bracketed max-over-ranks timing and the
fast_st leg's all-reduce of the flat gradient.  Two ranks share cuda:0 and exchange over
gloo (RCCL refuses two ranks on one device); on the 8-GPU node the same code runs one
rank per GPU over RCCL.  Reference: the static_train loop being sharded,
stransfer/network.py:651-770."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_bench_two_ranks_same_device():
    env = dict(os.environ, STX_BENCH_SAME_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--fast-steps", "2", "--gatys-run-iters", "10", "--skip-cpu",
           "--skip-infer"]
    # (the ranks' stderr goes to this test's own output: a hang or crash shows where)
    r = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, text=True, timeout=540)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints the line
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["devices"] == 1
    assert res["value"] > 0 and res["config"]["parallelism"] == "replicas2"
    fs = res["fast_st"]
    assert fs["parallelism"] == "dp2" and fs["global_batch"] == 2 * fs["per_gpu_batch"]
    assert fs["collective"] and "all_reduce" in fs["collective"]
    assert fs["value"] > 0
