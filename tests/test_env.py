"""Native synthetic microRTS env: tensor contracts of MicroRTSGridModeVecEnv."""
import numpy as np
import torch

from microbeast_amd.envs.synthetic import create_env
from microbeast_amd.ops.cell_head import OFFS, unpack_mask


def _rand_legal_actions(mask_bits, gen):
    mb = unpack_mask(mask_bits)
    n, S, _ = mb.shape
    a = torch.zeros(n, S, 7, dtype=torch.uint8)
    for k in range(7):
        seg = mb[..., OFFS[k]:OFFS[k + 1]].float() + 1e-6
        a[..., k] = torch.multinomial(seg.view(-1, seg.shape[-1]), 1, generator=gen).view(n, S)
    return a


def test_reference_api_shapes():
    env = create_env(8, 6, 2000)
    assert env.num_envs == 6 and env.height == 8
    assert env.observation_space.shape == (8, 8, 27)
    assert len(env.action_space.nvec) == 7 * 64 and env.action_space.shape == (448,)
    assert list(env.action_space.nvec[:7]) == [6, 4, 4, 4, 4, 7, 49]
    obs = env.reset()
    assert obs.shape == (6, 8, 8, 27) and obs.dtype == np.float32
    assert np.all(obs.sum(-1) == 5)  # 5 one-hot groups per cell
    m = env.get_action_mask()
    assert m.shape == (6, 64, 78)
    o, r, d, info = env.step(np.zeros((6, 448), dtype=np.int64))
    assert o.shape == obs.shape and r.shape == (6,) and d.shape == (6,) and len(info) == 6
    assert "\n" in env.render()


def test_compact_matches_dense_and_episodes_end():
    env = create_env(10, 8, 400, seed=3)
    S = 100
    obs = torch.zeros(8, S, dtype=torch.int32)
    mask = torch.zeros(8, S, 3, dtype=torch.int32)
    env.reset_compact(obs, mask)
    gen = torch.Generator().manual_seed(0)
    rew = torch.zeros(8)
    done = torch.zeros(8, dtype=torch.uint8)
    n_done = 0
    for _ in range(450):
        a = _rand_legal_actions(mask, gen)
        env.step_compact(a, obs, mask, rew, done)
        n_done += int(done.sum())
    assert n_done >= 8  # everything terminates by max_steps at the latest
    dense = env._dense_obs()
    bits = obs.numpy().view(np.uint32)
    rebuilt = ((bits[..., None] >> np.arange(27)) & 1).reshape(8, 10, 10, 27)
    assert np.array_equal(rebuilt.astype(np.float32), dense)
    dm = env.get_action_mask().astype(bool)
    assert np.array_equal(dm, unpack_mask(mask).numpy())
    eps = env.drain_episodes()
    assert len(eps) == n_done
    assert all(e[1] > 0 for e in eps)


def test_determinism():
    outs = []
    for _ in range(2):
        env = create_env(8, 4, 300, seed=11)
        obs = torch.zeros(4, 64, dtype=torch.int32)
        mask = torch.zeros(4, 64, 3, dtype=torch.int32)
        env.reset_compact(obs, mask)
        gen = torch.Generator().manual_seed(5)
        acc = []
        for _ in range(50):
            a = _rand_legal_actions(mask, gen)
            o, m, r, d = env.step_compact(a)
            acc.append(o.clone())
        outs.append(torch.stack(acc))
    assert torch.equal(outs[0], outs[1])


def test_masks_only_on_own_idle_units():
    env = create_env(16, 4, 2000, seed=2)
    obs, mask = env.reset_compact()
    mb = unpack_mask(mask)
    bits = obs.numpy().view(np.uint32)
    own = (bits >> 11) & 1  # owner plane "player 0"
    has_mask = mb.any(-1).numpy()
    assert np.all(own[has_mask] == 1)
    # every unit with a mask can at least no-op
    assert torch.all(mb[mb.any(-1)][:, 0])


def test_self_play_opponent_api():
    from microbeast_amd.envs.synthetic import SyntheticGridVecEnv
    env = SyntheticGridVecEnv(num_selfplay_envs=2, num_bot_envs=0, size=8, seed=1)
    env.reset_compact()
    o1 = torch.zeros(2, 64, dtype=torch.int32)
    m1 = torch.zeros(2, 64, 3, dtype=torch.int32)
    env._env.obs_p1(o1.data_ptr())
    env._env.mask_p1(m1.data_ptr())
    # player-1 view: its own units carry the "player 0" owner plane after mirroring
    b = o1.numpy().view(np.uint32)
    assert ((b >> 11) & 1).sum() > 0
    assert unpack_mask(m1).any()
    env._env.set_opponent_actions(torch.zeros(2, 64, 7, dtype=torch.uint8).data_ptr())
    env.step_compact(torch.zeros(2, 64, 7, dtype=torch.uint8))
