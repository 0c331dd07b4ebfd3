"""GPU actor engine end-to-end on the MI355X: slot alignment, learner update, publish."""
import pytest
import torch

from microbeast_amd.ops.cell_head import OFFS, unpack_mask

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["lanes1", "lanes2", "reference_keys"])
def test_engine_rollout_alignment_and_learn(cuda, variant):
    """Slot alignment / action legality / learn / publish through the captured-graph step
    forms: one and two lanes on the sparse row I/O; the reference buffer keys (dense code /
    action copies: their last_action rows are dense)."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    s, T = 8, 8
    lanes = 2 if variant == "lanes2" else 1

    def mk():
        return Agent((s, s, 27))

    torch.manual_seed(0)
    learner = Learner(mk(), LearnerHParams(), cuda)
    rt = GpuActorRuntime(mk, s, n_groups=2, envs_per_group=16, unroll=T, batch_slots=1,
                         device=cuda, n_threads=2, n_lanes=lanes,
                         reference_keys=variant == "reference_keys")
    assert not rt.fused_act  # 8x8: the captured-graph step
    assert rt.sparse_io == (variant != "reference_keys")
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
    assert rt.n_lanes == lanes
    for lane in rt.lanes:
        d = (lane["flat"].data - learner.flat.data).abs().max().item()
        assert d < 1e-2


@pytest.mark.parametrize("s", [8, 16])
def test_selfplay_league_engine(cuda, s):
    """Self-play groups: the opponent policy drives player 1 from league snapshots; its
    episodes come back tagged with the snapshot id; bot groups keep scripted opponents.
    16x16: both players on the fused acting step (sparse rows, the opponent's own weight
    block); 8x8: the captured-graph path."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime
    from microbeast_amd.runtime.league import League

    T, E = 8, 16

    def mk():
        return Agent((s, s, 27))

    torch.manual_seed(1)
    learner = Learner(mk(), LearnerHParams(), cuda)
    rt = GpuActorRuntime(mk, s, n_groups=2, envs_per_group=E, unroll=T, batch_slots=1,
                         device=cuda, n_threads=2, max_steps=12, selfplay_groups=1, n_lanes=2)
    assert rt.fused_act == (s == 16)
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


def test_engine_reference_keys(cuda):
    """Optional reference buffer keys (libs/utils.py:34-46) from the engine: ep_step counts
    1, 2, ... and restarts after done; ep_return is the running sum of reward; last_action[t]
    is the action of row t-1 (row 0: the previous slot's last action); policy_logits are the
    dense head's logits, whose masked log-softmax at the sampled action sums to the
    behaviour log-prob."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.cell_head import cell_head_torch
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    s, T = 8, 8

    def mk():
        m = Agent((s, s, 27))
        torch.nn.init.normal_(m.actor.weight, std=0.02)
        return m

    torch.manual_seed(0)
    learner = Learner(mk(), LearnerHParams(), cuda)
    rt = GpuActorRuntime(mk, s, n_groups=1, envs_per_group=16, unroll=T, batch_slots=1,
                         device=cuda, n_threads=2, max_steps=12, reference_keys=True,
                         policy_logits=True)
    rt.start(learner.flat)
    try:
        b1, sl1 = rt.get_batch()
        torch.cuda.synchronize()
        first = {k: v.clone() for k, v in b1.items()}
        rt.release(sl1)
        b2, sl2 = rt.get_batch()
        torch.cuda.synchronize()
        second = {k: v.clone() for k, v in b2.items()}
        rt.release(sl2)
    finally:
        rt.stop()
    for b in (first, second):
        st, ret = b["ep_step"][:T].cpu(), b["ep_return"][:T].cpu()
        rew, done = b["reward"][:T].cpu(), b["done"][:T].cpu().bool()
        for t in range(1, T):
            prev_done = done[t - 1]
            exp_step = torch.where(prev_done, torch.ones_like(st[t]), st[t - 1] + 1)
            assert torch.equal(st[t], exp_step)
            exp_ret = torch.where(prev_done, rew[t], ret[t - 1] + rew[t])
            torch.testing.assert_close(ret[t], exp_ret)
        assert torch.equal(b["last_action"][1:T], b["action"][:T - 1])
    assert torch.equal(second["last_action"][0], first["action"][T - 1])
    # behaviour log-prob from the emitted dense logits (fp32 torch semantics)
    lg = second["policy_logits"][:T].reshape(T * 16, -1).cpu()
    _, lp, _ = cell_head_torch(lg, second["mask"][:T].reshape(T * 16, s * s, 3).cpu(),
                               second["action"][:T].reshape(T * 16, s * s, 7).cpu())
    torch.testing.assert_close(lp, second["logp"][:T].reshape(-1).cpu(), rtol=2e-2, atol=5e-2)
