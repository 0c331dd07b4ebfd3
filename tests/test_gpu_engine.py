"""GPU actor engine end-to-end on the MI355X: slot alignment, learner update, publish."""
import pytest
import torch

from microbeast_amd.ops.cell_head import OFFS, unpack_mask

pytestmark = pytest.mark.gpu


def test_engine_rollout_alignment_and_learn(cuda):
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    s, T = 8, 8

    def mk():
        return Agent((s, s, 27))

    torch.manual_seed(0)
    learner = Learner(mk(), LearnerHParams(), cuda)
    rt = GpuActorRuntime(mk, s, n_groups=2, envs_per_group=16, unroll=T, batch_slots=1,
                         device=cuda, n_threads=2, n_lanes=2)
    rt.start(learner.flat)
    try:
        prev_last_obs = {}
        for it in range(6):
            batch, slots = rt.get_batch()
            torch.cuda.synchronize()
            obs, mask, act = batch["obs"], batch["mask"], batch["action"]
            # 5 hot planes per cell everywhere
            bits = obs.cpu().view(-1).numpy().view("uint32")
            assert set(int(bin(int(x)).count("1")) for x in bits[:5000]) == {5}
            # every sampled action component legal under the mask observed at the same t
            mb = unpack_mask(mask[:T].cpu())
            a = act[:T].cpu().long()
            for k in range(7):
                seg = mb[..., OFFS[k]:OFFS[k + 1]]
                has = seg.any(-1)
                ok = seg.gather(-1, a[..., k:k + 1]).squeeze(-1) | ~has
                assert bool(ok.all()), f"illegal action component {k}"
            losses = learner.learn(batch)
            rt.release(slots)
            assert rt.publish(learner.flat) in (True, False)
            assert torch.isfinite(losses).all()
        st = rt.stats()
        assert st["frames"] > 0 and st["gpu_steps"] > 0 and st["publishes"] >= 1
    finally:
        rt.stop()
    # every policy lane's inference weights track the learner after a publish
    torch.cuda.synchronize()
    assert rt.n_lanes == 2
    for lane in rt.lanes:
        d = (lane["flat"].data - learner.flat.data).abs().max().item()
        assert d < 1e-2


def test_selfplay_league_engine(cuda):
    """Self-play groups: the opponent graph drives player 1 from league snapshots; its
    episodes come back tagged with the snapshot id; bot groups keep scripted opponents."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime
    from microbeast_amd.runtime.league import League

    s, T, E = 8, 8, 16

    def mk():
        return Agent((s, s, 27))

    torch.manual_seed(1)
    learner = Learner(mk(), LearnerHParams(), cuda)
    rt = GpuActorRuntime(mk, s, n_groups=2, envs_per_group=E, unroll=T, batch_slots=1,
                         device=cuda, n_threads=2, max_steps=12, selfplay_groups=1, n_lanes=2)
    league = League(capacity=4, snapshot_every=2, eps=0.5, seed=3)
    sid0 = league.add_snapshot(learner.flat.data)
    rt.start(learner.flat, opponent_version=sid0)
    episodes = []
    try:
        for it in range(24):  # >= 12 slots of T=8 per group: every env ends >= 4 episodes
            batch, slots = rt.get_batch()
            losses = learner.learn(batch)
            rt.release(slots)
            rt.publish(learner.flat)
            league.maybe_snapshot(it + 1, learner.flat.data)
            sid = league.sample()
            if sid != league.current and rt.set_opponent(league.snapshot(sid), sid):
                league.current = sid
            assert torch.isfinite(losses).all()
            eps = rt.drain_episodes()
            league.record(eps)
            episodes += eps
        st = rt.stats()
    finally:
        rt.stop()
    assert st["opp_publishes"] >= 1 and st["opp_version"] in league.snaps
    sp = [e for e in episodes if e[2] >= E]    # second group = self-play envs
    bots = [e for e in episodes if e[2] < E]
    print("episodes", len(episodes), "selfplay", len(sp), "bots", len(bots), st)
    assert sp and bots
    assert all(e[4] >= 0 for e in sp) and all(e[4] < 0 for e in bots)
    assert sum(league.games.values()) == len(sp)
    # the opponent's weights are a league snapshot
    torch.cuda.synchronize()
    cur = st["opp_version"]
    assert torch.equal(rt.opp_flat.data, league.snapshot(cur)) or cur != league.current
