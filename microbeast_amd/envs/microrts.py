"""Optional adapter to the real gym-microRTS (Java engine through JPype).

The reference builds ``MicroRTSGridModeVecEnv`` directly (libs/utils.py:59-76).
gym-microrts is not installed in this image (no network), so this module is
gated: importing it without gym_microrts raises a clear error, and
``create_env(..., env="microrts")`` is the only entry point. Its outputs are
converted into the compact layout the rest of the framework uses.
"""
from __future__ import annotations

import numpy as np
import torch


def gym_microrts_available() -> bool:
    try:
        import gym_microrts  # noqa: F401
        return True
    except Exception:
        return False


class MicroRTSAdapter:
    """Wraps a MicroRTSGridModeVecEnv with the compact API of SyntheticGridVecEnv."""

    def __init__(self, env):
        self.env = env
        self.num_envs = env.num_envs
        self.height = self.width = env.height
        self.S = self.height * self.width
        self.observation_space = env.observation_space
        self.action_space = env.action_space
        self._eps = []
        self._ret = np.zeros(self.num_envs, np.float32)
        self._len = np.zeros(self.num_envs, np.int32)

    @staticmethod
    def _bits(obs: np.ndarray) -> torch.Tensor:
        n, h, w, p = obs.shape
        wts = (1 << np.arange(p, dtype=np.int64))
        v = ((obs.reshape(n, h * w, p) > 0.5).astype(np.int64) * wts).sum(-1)
        return torch.from_numpy(v.astype(np.int32))

    @staticmethod
    def _mask_bits(mask: np.ndarray, n: int, S: int) -> torch.Tensor:
        from ..ops.cell_head import pack_mask

        return pack_mask(torch.from_numpy(mask.reshape(n, S, 78).astype(bool)))

    def reset_compact(self, obs=None, mask=None):
        o = self._bits(self.env.reset())
        m = self._mask_bits(self.env.get_action_mask(), self.num_envs, self.S)
        if obs is not None:
            obs.copy_(o)
            mask.copy_(m)
            return obs, mask
        return o, m

    def step_compact(self, actions, obs=None, mask=None, reward=None, done=None):
        a = actions.reshape(self.num_envs, -1).long().numpy()
        o, r, d, _ = self.env.step(a)
        self._ret += r
        self._len += 1
        for i in np.where(d)[0]:
            self._eps.append((float(self._ret[i]), int(self._len[i]), int(i), -1))
            self._ret[i] = 0
            self._len[i] = 0
        ob = self._bits(o)
        mk = self._mask_bits(self.env.get_action_mask(), self.num_envs, self.S)
        rw = torch.from_numpy(np.asarray(r, np.float32))
        dn = torch.from_numpy(np.asarray(d).astype(np.uint8))
        if obs is None:
            return ob, mk, rw, dn
        obs.copy_(ob)
        mask.copy_(mk)
        reward.copy_(rw)
        done.copy_(dn)
        return obs, mask, reward, done

    def drain_episodes(self):
        e, self._eps = self._eps, []
        return e

    def close(self):
        self.env.close()


# --opponents names (config.py, the native stand-in's bots) -> gym_microrts.microrts_ai members
# (reference libs/utils.py:69-72 builds ai2s from coacAI, randomBiasedAI, lightRushAI,
# workerRushAI); microrts_ai names pass through unchanged
MICRORTS_AI = {"coac": "coacAI", "random_biased": "randomBiasedAI", "light_rush": "lightRushAI",
               "worker_rush": "workerRushAI", "passive": "passiveAI", "random": "randomAI"}
REFERENCE_AI2S = ["coacAI"] * 3 + ["randomBiasedAI", "lightRushAI", "workerRushAI"]


def microrts_ai_names(opponents) -> list[str]:
    return [MICRORTS_AI.get(n, n) for n in (opponents or REFERENCE_AI2S)]


def create_microrts_env(size, n_envs, max_steps, opponents=None, reward_weight=None):
    """The reference's create_env (libs/utils.py:59-76) on the real gym-microRTS."""
    if not gym_microrts_available():
        raise RuntimeError("env=microrts needs gym-microrts (Java microRTS); it is not installed. "
                           "Use --env synthetic.")
    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    names = microrts_ai_names(opponents)
    missing = [n for n in names if not hasattr(microrts_ai, n)]
    if missing:
        raise ValueError(f"gym_microrts.microrts_ai has no {missing} (--opponents)")
    ai2s = [getattr(microrts_ai, n) for n in names][:n_envs]
    while len(ai2s) < n_envs:
        ai2s.append(ai2s[len(ai2s) % len(names)])
    env = MicroRTSGridModeVecEnv(
        num_selfplay_envs=0, num_bot_envs=n_envs, max_steps=max_steps, render_theme=2, ai2s=ai2s,
        map_paths=[f"maps/{size}x{size}/basesWorkers{size}x{size}.xml"],
        reward_weight=np.array(reward_weight or [10.0, 1.0, 1.0, 0.2, 1.0, 4.0]))
    return MicroRTSAdapter(env)
