"""Reference-shaped CPU runtime end to end: BASELINE config 1 plumbing (4x4, 2 CPU actors,
CPU learner), CSV logs, checkpoint + resume, watchdog under fault injection, --test eval."""
import os

import pytest
import torch

from microbeast_amd.config import parse_flags
from microbeast_amd.utils.checkpoint import load_checkpoint

pytestmark = pytest.mark.slow


def _flags(tmp, *extra):
    return parse_flags(["--exp_name", "plumb", "--env_size", "4", "--n_actors", "2", "--n_envs",
                        "4", "--unroll_length", "8", "--batch_size", "2", "--savedir", str(tmp),
                        "--device", "cpu", "--quiet", "--checkpoint_every", "2", *extra],
                       interactive=False)


def test_plumbing_resume_and_eval(tmp_path):
    from microbeast_amd.evaluate import evaluate
    from microbeast_amd.train import train
    out = train(_flags(tmp_path, "--max_updates", "4"))
    assert out["updates"] == 4 and out["steps"] == 4 * 2 * 4 * 8
    ck = load_checkpoint(os.path.join(tmp_path, "plumb.ckpt"))
    assert ck["n_update"] == 4
    losses = open(tmp_path / "plumbLosses.csv").read().splitlines()
    assert len(losses) == 5
    out = train(_flags(tmp_path, "--max_updates", "6", "--resume"))
    assert out["updates"] == 6
    assert len(open(tmp_path / "plumbLosses.csv").read().splitlines()) == 7  # appended
    res = evaluate(_flags(tmp_path, "--eval_episodes", "3", "--max_episode_steps", "200"))
    assert res["episodes"] == 3 and os.path.exists(res["csv"])


def test_watchdog_respawns_killed_actors(tmp_path):
    from microbeast_amd.train import train
    out = train(_flags(tmp_path, "--max_updates", "6", "--fault_inject_every", "2",
                       "--actor_restarts", "10", "--batch_timeout", "120"))
    assert out["updates"] == 6


def test_profiler_trace_written(tmp_path):
    from microbeast_amd.train import train
    out = train(_flags(tmp_path, "--max_updates", "6", "--profile_updates", "2"))
    assert out["updates"] == 6
    assert os.path.getsize(tmp_path / "plumb_trace.json") > 0
    assert "Name" in open(tmp_path / "plumb_profile.txt").read()
