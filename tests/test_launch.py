"""One-process-per-GPU launcher and rank placement (parallel/launch.py).

* the core-placement rule: disjoint whole-core shares of the GPU's NUMA node, SMT
  siblings kept together, quota-aware fallback;
* ``microbeast.py --nproc_per_node 2`` with no torchrun environment launches 2
  data-parallel ranks itself (gloo, CPU): both ranks' episodes reach rank 0's CSV over
  the host group, one Losses.csv row per update with the phase / lag columns."""
import csv
import os
import subprocess
import sys

import pytest

from microbeast_amd.parallel import launch as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_cpulist():
    assert L.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert L.parse_cpulist("") == []


def test_split_cores_disjoint_and_covering():
    cores = [[i, i + 64] for i in range(48)]  # 48 cores with SMT siblings i, i+64
    parts = [L.split_cores(cores, 4, i) for i in range(4)]
    flat = [c for p in parts for c in p]
    assert sorted(flat) == sorted(c for core in cores for c in core)
    assert len(set(flat)) == len(flat)
    for p in parts:  # siblings stay together
        assert all((c + 64 in p) for c in p if c < 64)


def test_plan_affinity_numa_split(monkeypatch):
    # 2 NUMA nodes x 8 cores (no SMT info -> 1 cpu per core); GPUs 0-3 on node 0, 4-7 on 1
    monkeypatch.setattr(L, "_read", lambda path: None)
    allowed = list(range(16))
    node_of_rank = [0, 0, 0, 0, 1, 1, 1, 1]
    cpus = {0: list(range(8)), 1: list(range(8, 16))}
    got = [L.plan_affinity(r, 8, allowed, node_of_rank, cpus) for r in range(8)]
    assert got[0] == [0, 1] and got[3] == [6, 7] and got[4] == [8, 9] and got[7] == [14, 15]
    # node share below the quota share: fall back to the plain split of allowed CPUs
    one = L.plan_affinity(0, 1, list(range(64)), [0], {0: [0, 1, 2, 3]}, min_cpus=16)
    assert len(one) == 64
    # unknown topology
    assert L.plan_affinity(1, 2, allowed, [-1, -1], {}) == list(range(8, 16))


def test_relaunch_noop_inside_torchrun(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert L.relaunch(2, [], script="x.py") is None
    monkeypatch.delenv("WORLD_SIZE")
    assert L.relaunch(1, [], script="x.py") is None


def test_relaunch_refuses_missing_gpus(monkeypatch):
    import torch
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert L.relaunch(4, [], script="x.py") == 2


@pytest.mark.slow
def test_cli_self_launches_two_cpu_ranks(tmp_path):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "microbeast.py"), "--exp_name", "dp2",
           "--nproc_per_node", "2", "--device", "cpu", "--runtime", "mono", "--env_size", "4",
           "--n_actors", "1", "--n_envs", "4", "--unroll_length", "8", "--batch_size", "1",
           "--max_updates", "3", "--max_episode_steps", "20", "--savedir", str(tmp_path),
           "--quiet", "--actor_inference", "local"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=600, stdin=subprocess.DEVNULL)
    assert r.returncode == 0, r.stderr[-4000:]
    with open(tmp_path / "dp2Losses.csv") as f:
        rows = list(csv.DictReader(f))
    assert [int(x["update"]) for x in rows] == [1, 2, 3]
    assert all(x["policy_lag"] == "-1" for x in rows) and "fwd_ms" in rows[0]
    assert int(rows[-1]["frames"]) == 3 * 2 * 1 * 4 * 8  # both ranks' frames counted
    with open(tmp_path / "dp2.csv") as f:
        eps = list(csv.DictReader(f))
    # 20-step episodes on 4 envs per rank: both ranks' env index ranges show up
    idx = {int(e["env_index"]) for e in eps}
    assert eps and min(idx) < 4 <= max(idx)
