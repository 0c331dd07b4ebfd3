"""Real gym-microRTS adapter (envs/microrts.py) against a stub ``gym_microrts`` module.

gym-microrts (Java microRTS through JPype) is not installable here, so real-env parity stays
unpinned; what is pinned is the constructor call the reference makes (libs/utils.py:59-76):
0 self-play envs, n bot envs, max_steps, render_theme 2, ai2s = 3 x coacAI, randomBiasedAI,
lightRushAI, workerRushAI (the --opponents names mapped to microrts_ai members), the
basesWorkers map path and the reward weights -- and the compact conversion of its outputs."""
import sys
import types

import numpy as np
import pytest
import torch


class _StubVecEnv:
    calls = []

    def __init__(self, **kw):
        _StubVecEnv.calls.append(kw)
        self.num_envs = kw["num_bot_envs"]
        self.height = 8
        self.observation_space = types.SimpleNamespace(shape=(8, 8, 27))
        self.action_space = types.SimpleNamespace(nvec=np.array([6, 4, 4, 4, 4, 7, 49] * 64),
                                                  shape=(64 * 7,))
        self.rng = np.random.default_rng(0)

    def _obs(self):
        o = np.zeros((self.num_envs, 8, 8, 27), np.int32)
        for g0, n in ((0, 5), (5, 5), (10, 3), (13, 8), (21, 6)):  # 5 one-hot groups
            idx = self.rng.integers(0, n, size=(self.num_envs, 8, 8))
            np.put_along_axis(o[..., g0:g0 + n], idx[..., None], 1, axis=-1)
        return o

    def reset(self):
        return self._obs()

    def get_action_mask(self):
        m = np.zeros((self.num_envs, 64, 78), np.int32)
        m[:, 9, 0] = 1
        m[:, 9, 7] = 1
        return m.reshape(self.num_envs, -1)

    def step(self, a):
        assert a.shape == (self.num_envs, 64 * 7)
        d = np.zeros(self.num_envs, bool)
        d[0] = True
        return self._obs(), np.ones(self.num_envs, np.float32), d, [{}] * self.num_envs

    def close(self):
        pass


@pytest.fixture
def stub_gym_microrts(monkeypatch):
    pkg = types.ModuleType("gym_microrts")
    ai = types.ModuleType("gym_microrts.microrts_ai")
    for n in ("coacAI", "randomBiasedAI", "lightRushAI", "workerRushAI", "passiveAI", "randomAI"):
        setattr(ai, n, f"<{n}>")
    envs = types.ModuleType("gym_microrts.envs")
    vec = types.ModuleType("gym_microrts.envs.vec_env")
    vec.MicroRTSGridModeVecEnv = lambda **kw: _StubVecEnv(**kw)
    pkg.microrts_ai = ai
    pkg.envs = envs
    envs.vec_env = vec
    for name, mod in (("gym_microrts", pkg), ("gym_microrts.microrts_ai", ai),
                      ("gym_microrts.envs", envs), ("gym_microrts.envs.vec_env", vec)):
        monkeypatch.setitem(sys.modules, name, mod)
    _StubVecEnv.calls.clear()
    return _StubVecEnv


def test_create_env_matches_reference_constructor(stub_gym_microrts):
    from microbeast_amd.config import Flags
    from microbeast_amd.envs.synthetic import create_env

    flags = Flags()  # default --opponents = the reference bot mix in our names
    env = create_env(8, 6, 2000, env="microrts", opponents=flags.opponent_list(),
                     reward_weight=flags.reward_weights())
    (kw,) = stub_gym_microrts.calls
    assert kw["num_selfplay_envs"] == 0 and kw["num_bot_envs"] == 6
    assert kw["max_steps"] == 2000 and kw["render_theme"] == 2
    assert kw["ai2s"] == ["<coacAI>"] * 3 + ["<randomBiasedAI>", "<lightRushAI>",
                                              "<workerRushAI>"]
    assert kw["map_paths"] == ["maps/8x8/basesWorkers8x8.xml"]
    assert np.allclose(kw["reward_weight"], [10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    # more envs than opponents: the bot list repeats (the reference has exactly 6)
    create_env(8, 8, 500, env="microrts", opponents=["coac", "worker_rush"])
    assert stub_gym_microrts.calls[-1]["ai2s"] == ["<coacAI>", "<workerRushAI>"] * 4


def test_adapter_compact_outputs(stub_gym_microrts):
    from microbeast_amd.envs.synthetic import create_env
    from microbeast_amd.ops.cell_head import unpack_mask

    env = create_env(8, 4, 100, env="microrts")
    obs, mask = env.reset_compact()
    assert obs.shape == (4, 64) and obs.dtype == torch.int32
    bits = obs.numpy().view(np.uint32)
    assert set(int(bin(int(x)).count("1")) for x in bits.ravel()) == {5}
    mb = unpack_mask(mask)
    assert mb.shape == (4, 64, 78) and bool(mb[:, 9, 0].all()) and int(mb.sum()) == 8
    o, m, r, d = env.step_compact(torch.zeros(4, 64, 7, dtype=torch.uint8))
    assert float(r.sum()) == 4.0 and int(d[0]) == 1
    eps = env.drain_episodes()
    assert len(eps) == 1 and eps[0][0] == 1.0 and eps[0][1] == 1


def test_unknown_opponent_is_an_error(stub_gym_microrts):
    from microbeast_amd.envs.synthetic import create_env
    with pytest.raises(ValueError, match="microrts_ai"):
        create_env(8, 2, 100, env="microrts", opponents=["no_such_bot"])
