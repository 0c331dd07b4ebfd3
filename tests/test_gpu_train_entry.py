"""The user-facing GPU entry point ``microbeast.py --runtime gpu`` end to end on the MI355X
(reference microbeast.py:109-278 ``train()`` / ``main()``): rank-0 CSVs in the reference
formats, checkpoint, ``--resume`` (CSV append, step / update restore), ``--test``
evaluation on the GPU, the self-play league's state through a checkpoint, and a
short-budget run whose episode return and win rate must improve (the reference's logged
runs stay flat: experiments/5_ener/5_enero.csv)."""
import csv
import os

import pytest
import torch

from microbeast_amd.cli import main
from microbeast_amd.utils.checkpoint import load_checkpoint

pytestmark = pytest.mark.gpu


def _args(tmp, name, *extra):
    return ["--exp_name", name, "--runtime", "gpu", "--env_size", "8", "--groups", "2",
            "--envs_per_group", "32", "--unroll_length", "8", "--batch_size", "1",
            "--savedir", str(tmp), "--quiet", "--max_episode_steps", "10", *extra]


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def test_gpu_train_checkpoint_resume_and_eval(cuda, tmp_path):
    assert main(_args(tmp_path, "g", "--max_updates", "4", "--checkpoint_every", "2")) == 0
    ck = load_checkpoint(os.path.join(tmp_path, "g.ckpt"))
    frames = 32 * 8
    assert ck["n_update"] == 4 and ck["step"] == 4 * frames
    loss = _rows(tmp_path / "gLosses.csv")
    assert [int(r["update"]) for r in loss] == [1, 2, 3, 4]
    assert all(int(r["policy_lag"]) >= 0 for r in loss)
    assert all(float(r["fwd_ms"]) > 0 for r in loss[1:])  # HIP-event phase split, read late
    eps = _rows(tmp_path / "g.csv")
    assert eps and set(eps[0]) >= {"Return", "steps"}
    w0 = ck["model_state_dict"]["actor.weight"].clone()
    assert main(_args(tmp_path, "g", "--max_updates", "6", "--resume")) == 0
    ck2 = load_checkpoint(os.path.join(tmp_path, "g.ckpt"))
    assert ck2["n_update"] == 6 and ck2["step"] == 6 * frames
    assert not torch.equal(ck2["model_state_dict"]["actor.weight"], w0)  # it kept learning
    assert ck2["optimizer_state_dict"]["step"] == 6  # Adam moments / step restored, not reset
    loss = _rows(tmp_path / "gLosses.csv")
    assert [int(r["update"]) for r in loss] == [1, 2, 3, 4, 5, 6]  # appended, no new header
    assert main(_args(tmp_path, "g", "--test", "--eval_episodes", "3", "--n_envs", "3")) == 0
    ev = _rows(tmp_path / "g_eval.csv")
    assert len(ev) == 3


def test_gpu_selfplay_league_survives_resume(cuda, tmp_path):
    a = ["--self_play", "--selfplay_groups", "1", "--league_update_every", "1",
         "--league_size", "4"]
    assert main(_args(tmp_path, "sp", "--max_updates", "3", *a)) == 0
    ck = load_checkpoint(os.path.join(tmp_path, "sp.ckpt"))
    lg = ck["league"]
    n0 = len(lg["snaps"])
    assert n0 >= 2 and lg["next_id"] == 4  # initial + a snapshot every update (capacity 4)
    assert main(_args(tmp_path, "sp", "--max_updates", "5", "--resume", *a)) == 0
    ck2 = load_checkpoint(os.path.join(tmp_path, "sp.ckpt"))
    lg2 = ck2["league"]
    # the pool, ids and results continued from the checkpoint instead of restarting
    assert ck2["n_update"] == 5 and lg2["next_id"] == 6 and len(lg2["snaps"]) == 4
    assert sum(lg2["games"].values()) >= sum(lg["games"].values())
    eps = _rows(tmp_path / "sp.csv")
    assert any(int(e["opponent"]) >= 0 for e in eps)  # league-tagged self-play episodes


def test_gpu_training_improves_return_and_win_rate(cuda, tmp_path):
    """8x8 against the passive bot, 1500 updates of 16K frames (~15 s): the second half's
    episodes must beat the first 15 % on win rate and on return per step. (Mean episode return
    is not monotone here: with the microRTS unit timings the learned policy wins in fewer steps,
    so it collects fewer shaped harvest / production rewards per episode; measured 42.7 -> 33.9
    while the win rate went 0.82 -> 1.00.)"""
    assert main(["--exp_name", "learn", "--runtime", "gpu", "--env_size", "8", "--opponents",
                 "passive", "--groups", "2", "--envs_per_group", "256", "--unroll_length", "64",
                 "--batch_size", "1", "--max_updates", "1500", "--max_episode_steps", "400",
                 "--savedir", str(tmp_path), "--quiet", "--log_every", "50",
                 "--checkpoint_every", "0"]) == 0
    eps = _rows(tmp_path / "learn.csv")
    n = len(eps)
    assert n > 2000
    first, last = eps[:int(0.15 * n)], eps[n // 2:]

    def stats(rows):
        ret = sum(float(r["Return"]) for r in rows)
        steps = sum(int(r["steps"]) for r in rows)
        win = sum(r["winner"] == "0" for r in rows) / len(rows)
        return ret / len(rows), ret / steps, win

    (r0, q0, w0), (r1, q1, w1) = stats(first), stats(last)
    print(f"return {r0:.1f} -> {r1:.1f}, per step {q0:.3f} -> {q1:.3f}, win rate {w0:.3f} -> "
          f"{w1:.3f} over {n} episodes")
    assert q1 > 1.1 * q0 and w1 > w0


def test_gpu_engine_fault_injection_recovers(cuda, tmp_path):
    """SURVEY §5.3 on the flagship runtime: an env worker that throws stops the native
    engine (instead of terminating the process); train() rebuilds the actor side from the
    live learner and keeps going, bounded by --actor_restarts."""
    from microbeast_amd.config import parse_flags
    from microbeast_amd.train import train
    out = train(parse_flags(_args(tmp_path, "fi", "--max_updates", "6", "--fault_inject_every",
                                  "2", "--actor_restarts", "5", "--batch_timeout", "120"),
                            interactive=False))
    assert out["updates"] == 6 and out["engine_restarts"] >= 2
    loss = _rows(tmp_path / "fiLosses.csv")
    assert [int(r["update"]) for r in loss] == [1, 2, 3, 4, 5, 6]


def test_gpu_engine_failure_surfaces_without_restarts(cuda, tmp_path):
    from microbeast_amd.config import parse_flags
    from microbeast_amd.runtime.gpu_actors import EngineFailure
    from microbeast_amd.train import train
    with pytest.raises(EngineFailure, match="injected env-worker fault"):
        train(parse_flags(_args(tmp_path, "fx", "--max_updates", "6", "--fault_inject_every",
                                "2", "--actor_restarts", "0", "--batch_timeout", "120"),
                          interactive=False))


def test_engine_restart_frees_the_old_runtime_first(cuda):
    """train.restart_runtime: the failed runtime's HBM (rollout slots, I/O, graphs) is released
    before the new one is allocated, so a restart peaks at about ONE runtime's footprint, and
    the new engine's slots carry the learner's current update (policy lag 0, not n_update)."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime
    from microbeast_amd.train import restart_runtime

    torch.cuda.synchronize()
    learner = Learner(Agent((8, 8, 27)), LearnerHParams(), cuda)

    def mk():
        return GpuActorRuntime(lambda: Agent((8, 8, 27)), 8, 2, 256, 16, 1, cuda, n_threads=2)

    torch.cuda.synchronize()
    m0 = torch.cuda.memory_allocated()
    rt = mk()
    rt.start(learner.flat)
    batch, slots = rt.get_batch(timeout=120)
    rt.release(slots)
    del batch
    torch.cuda.synchronize()
    m1 = torch.cuda.memory_allocated()
    one = m1 - m0
    torch.cuda.reset_peak_memory_stats()
    rt = restart_runtime(rt, mk, learner.flat, 7)
    torch.cuda.synchronize()
    peak, m2 = torch.cuda.max_memory_allocated(), torch.cuda.memory_allocated()
    print(f"runtime {one / 2**20:.1f} MiB, after restart {(m2 - m0) / 2**20:.1f} MiB, "
          f"restart peak {(peak - m0) / 2**20:.1f} MiB")
    try:
        assert abs(m2 - m1) < 0.1 * one
        assert peak - m0 < 1.3 * one
        batch, slots = rt.get_batch(timeout=120)
        assert rt.policy_lag(slots, 7) == 0
        rt.release(slots)
    finally:
        rt.stop()


def test_gpu_fused_16x16_training_improves(cuda, tmp_path):
    """the headline acting path learns -- 16x16 through the fused two-launch
    policy step (wave-owned trunk launch A with bitmap rows, head launch B, 2 policy lanes) and
    the learner's head_score / head_bwd2 epilogues, against the passive bot: the second half's
    episodes must beat the first 15 % on return per step and on win rate."""
    from microbeast_amd.config import parse_flags
    from microbeast_amd.train import train
    out = train(parse_flags(["--exp_name", "l16", "--runtime", "gpu", "--env_size", "16",
                             "--opponents", "passive", "--groups", "2", "--envs_per_group",
                             "1024", "--policy_lanes", "2", "--unroll_length", "32",
                             "--batch_size", "1", "--max_updates", "700",
                             "--max_episode_steps", "300", "--savedir", str(tmp_path),
                             "--quiet", "--log_every", "50", "--checkpoint_every", "0"],
                            interactive=False))
    assert out["fused_act"], "the 16x16 run did not take the fused acting step"
    eps = _rows(tmp_path / "l16.csv")
    n = len(eps)
    assert n > 2000
    first, last = eps[:int(0.15 * n)], eps[n // 2:]

    def stats(rows):
        ret = sum(float(r["Return"]) for r in rows)
        steps = sum(int(r["steps"]) for r in rows)
        win = sum(r["winner"] == "0" for r in rows) / len(rows)
        return ret / len(rows), ret / steps, win

    (r0, q0, w0), (r1, q1, w1) = stats(first), stats(last)
    print(f"16x16 fused: return {r0:.2f} -> {r1:.2f}, per step {q0:.4f} -> {q1:.4f}, win rate "
          f"{w0:.3f} -> {w1:.3f} over {n} episodes, {out['mean_fps']:.0f} frames/s")
    assert r1 > r0 and q1 > 1.1 * q0 and w1 >= w0
