"""Multi-rank bench path on the single-GPU box: 2 DP ranks sharing cuda:0 over gloo
(RCCL refuses two ranks on one device). Exercises torchrun env parsing, broadcast,
bucketed all-reduce of CUDA grads, barriers, MAX-time reduction and rank-0 JSON."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_one_gpu(cuda):
    env = dict(os.environ, MBK_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--groups", "2", "--envs_per_group", "128",
           "--unroll", "16", "--threads", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["config"]["global_batch"] == 2 * 128 * 16
