"""Reference-shaped CPU runtime end to end: BASELINE config 1 plumbing (4x4, 2 CPU actors,
CPU learner), CSV logs, checkpoint + resume, watchdog under fault injection, --test eval."""
import os
import time

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


def test_inference_server_mode_cpu(tmp_path):
    """Actors get their actions from the batched policy server in the learner process
    (the GPU-learner path, exercised here on a CPU device with the same protocol)."""
    from microbeast_amd.train import train
    out = train(_flags(tmp_path, "--max_updates", "4", "--n_actors", "3",
                       "--actor_inference", "server", "--inference_wait_ms", "5"))
    assert out["updates"] == 4 and out["steps"] == 4 * 2 * 4 * 8
    assert len(open(tmp_path / "plumbLosses.csv").read().splitlines()) == 5


def test_inference_server_survives_actor_respawn(tmp_path):
    """Watchdog respawns killed actors; request sequence numbers keep a respawned actor
    from consuming a reply addressed to the process it replaced."""
    from microbeast_amd.train import train
    out = train(_flags(tmp_path, "--max_updates", "6", "--fault_inject_every", "2",
                       "--actor_restarts", "10", "--batch_timeout", "120",
                       "--actor_inference", "server"))
    assert out["updates"] == 6


def test_inference_server_batches_and_publishes():
    """Direct protocol test: concurrent clients are served in shared batches, replies
    match a local policy call on the same weights, and a publish lands before the next
    batch."""
    import threading

    from microbeast_amd.envs.synthetic import create_env
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.inference import InferenceServer

    s, n, A = 4, 3, 4
    torch.manual_seed(0)
    ref = Agent((s, s, 27))
    srv = InferenceServer(lambda: Agent((s, s, 27)), A, n, s, "cpu", max_wait_ms=50.0)
    try:
        srv.publish(_flat_of(ref))
        srv.start()
        clients = [srv.client(i) for i in range(A)]
        for i, c in enumerate(clients):
            env = create_env(s, n, 100, seed=10 + i)
            env.reset_compact(c.obs, c.mask)
        got = [None] * A

        def run(i):
            r = clients[i].act(timeout=30)
            got[i] = None if r is None else tuple(x.clone() for x in r)

        th = [threading.Thread(target=run, args=(i,)) for i in range(A)]
        for t in th:
            t.start()
        for t in th:
            t.join(30)
        assert all(g is not None for g in got)
        # (the server books a batch's statistics after replying: under a loaded CPU the
        # clients can return first)
        deadline = time.time() + 5.0
        while srv.stats()["mean_batch_actors"] == 0.0 and time.time() < deadline:
            time.sleep(0.01)
        assert srv.stats()["mean_batch_actors"] > 1.0  # dynamic batching happened
        for i, (a, lp, v) in enumerate(got):
            _, _, v_ref = ref.act(clients[i].obs, clients[i].mask,
                                  generator=torch.Generator().manual_seed(0))
            torch.testing.assert_close(v, v_ref.float(), rtol=1e-4, atol=1e-4)
            assert a.shape == (n, s * s, 7) and lp.shape == (n,)
        # a publish (all-zero weights -> value = 0) is in place for the next batch
        srv.publish(torch.zeros_like(_flat_of(ref)))
        a, lp, v = clients[0].act(timeout=30)
        assert float(v.abs().max()) == 0.0
    finally:
        srv.stop()


def _flat_of(model):
    from microbeast_amd.ops.optim import FlatParams
    import copy
    return FlatParams(copy.deepcopy(model), "cpu").data
