"""Multi-rank bench path on the single-GPU box: ``bench.py --gpus 2`` with no torchrun
environment launches its 2 DP ranks itself (parallel/launch.py); ``--oversubscribe`` lets
them share cuda:0 over gloo (RCCL refuses two ranks on one device). Exercises the
self-launch, torchrun env parsing, rank pinning, broadcast, bucketed all-reduce of CUDA
grads, barriers, MAX-time reduction and rank-0 JSON. (RCCL itself: test_gpu_dist_rccl.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_bench_two_ranks_one_gpu(cuda, scaling):
    """weak: each rank 2 x 128 envs, global batch 2 x (128 x 16); strong: the 1-GPU problem
    (2 x 128 envs, 128 x 16 frames per update) split over the 2 ranks."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--oversubscribe",
           "--steps", "3", "--warmup", "1", "--groups", "2", "--envs_per_group", "128",
           "--unroll", "16", "--threads", "2", "--scaling", scaling]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["scaling"] == scaling and out["value"] > 0
    if scaling == "weak":
        assert out["config"]["global_batch"] == 2 * 128 * 16
        assert out["config"]["envs_per_gpu"] == 2 * 128
    else:
        assert out["config"]["global_batch"] == 128 * 16
        assert out["config"]["envs_per_gpu"] == 2 * 64
        # the halved groups step on concurrent policy lanes (not one latency-bound lane)
        assert out["config"]["policy_lanes"] == 2
    print(json.dumps(out))
    assert out["policy_lag_updates"]["max"] >= 0
    assert set(out["learner_phase_ms_rank0"]) >= {"fwd", "bwd", "allreduce", "optim"}
    per = out["actor_stats_per_rank"]  # every rank's actor side, gathered to rank 0
    assert [r["rank"] for r in per] == [0, 1]
    assert all(r["frames_stepped_per_s"] > 0 and r["cpus_per_rank"] >= 1 for r in per)


def test_bench_refuses_more_gpus_than_visible(cuda):
    import torch
    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "1"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "visible GPUs" in r.stderr
