"""gym-microRTS GridMode vec-env API over the native synthetic simulator.

Mirrors the surface of ``MicroRTSGridModeVecEnv`` the reference uses
(libs/utils.py:64-75; env_packer.py:22-111; microbeast.py:144-146):
``num_envs``, ``height``/``width``, ``observation_space.shape`` =
(h, w, 27), ``action_space.nvec`` = [6,4,4,4,4,7,49] * h*w and
``action_space.shape`` = (7*h*w,), ``reset() -> obs``, ``step(action) ->
(obs, reward, done, infos)``, ``get_action_mask()``, ``render()``, ``close()``.

Two I/O flavours:
* reference (dense numpy): obs float32 (n,h,w,27), mask uint8 (n, h*w, 78);
* compact (torch, zero-copy into caller buffers): obs uint32 bit planes
  (n, h*w), mask 3 x uint32 bits per cell, actions uint8 (n, h*w, 7).
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import torch

from .. import _native as N

BOT_IDS = {"coac": 0, "random_biased": 1, "light_rush": 2, "worker_rush": 3, "passive": 4,
           "random": 5,
           # reference opponent names (gym_microrts.microrts_ai)
           "coacAI": 0, "randomBiasedAI": 1, "lightRushAI": 2, "workerRushAI": 3,
           "passiveAI": 4, "randomAI": 5}
NVEC_CELL = [6, 4, 4, 4, 4, 7, 49]
REFERENCE_OPPONENTS = ["coacAI", "coacAI", "coacAI", "randomBiasedAI", "lightRushAI",
                       "workerRushAI"]


class SyntheticGridVecEnv:
    def __init__(self, num_selfplay_envs: int = 0, num_bot_envs: int = 6, max_steps: int = 2000,
                 render_theme: int = 2, ai2s=None, map_paths=None, reward_weight=None,
                 size: int | None = None, seed: int = 0, env_index_base: int = 0):
        if size is None:
            size = 8
            if map_paths:
                # "maps/{s}x{s}/basesWorkers{s}x{s}.xml"
                tok = str(map_paths[0]).split("/")[-2]
                size = int(tok.split("x")[0])
        n = num_bot_envs + num_selfplay_envs
        bots = [BOT_IDS[b] if isinstance(b, str) else int(b)
                for b in (ai2s or REFERENCE_OPPONENTS)]
        rw = list(reward_weight) if reward_weight is not None else [10.0, 1.0, 1.0, 0.2, 1.0, 4.0]
        self._env = N.runtime().VecEnv(size, n, max_steps, seed, bots, [float(x) for x in rw],
                                       env_index_base)
        if num_selfplay_envs:
            self._env.set_external_opponent(True)
        self.num_envs = n
        self.height = self.width = size
        self.S = size * size
        self.observation_space = SimpleNamespace(shape=(size, size, 27))
        self.action_space = SimpleNamespace(nvec=np.array(NVEC_CELL * self.S),
                                            shape=(7 * self.S,))
        self._obs = torch.zeros(n, self.S, dtype=torch.int32)
        self._mask = torch.zeros(n, self.S, 3, dtype=torch.int32)
        self._rew = torch.zeros(n, dtype=torch.float32)
        self._done = torch.zeros(n, dtype=torch.uint8)
        self._act = torch.zeros(n, self.S, 7, dtype=torch.uint8)
        self._closed = False

    # ------------------------------------------------------------ compact API
    def reset_compact(self, obs: torch.Tensor | None = None, mask: torch.Tensor | None = None):
        obs = self._obs if obs is None else obs
        mask = self._mask if mask is None else mask
        self._env.reset(obs.data_ptr(), mask.data_ptr())
        if obs is not self._obs:
            self._obs.copy_(obs)
            self._mask.copy_(mask)
        return obs, mask

    def step_compact(self, actions: torch.Tensor, obs=None, mask=None, reward=None, done=None):
        """actions uint8 (n, h*w, 7) contiguous CPU; outputs written in place."""
        a = actions.contiguous()
        obs = self._obs if obs is None else obs
        mask = self._mask if mask is None else mask
        reward = self._rew if reward is None else reward
        done = self._done if done is None else done
        self._env.step(a.data_ptr(), obs.data_ptr(), mask.data_ptr(), reward.data_ptr(),
                       done.data_ptr())
        if obs is not self._obs:
            self._obs.copy_(obs)
            self._mask.copy_(mask)
        return obs, mask, reward, done

    def drain_episodes(self):
        """[(return, length, env_index, winner)] of episodes finished since the last call."""
        return self._env.drain_episodes()

    # ------------------------------------------------------------ reference API
    def reset(self):
        self.reset_compact()
        return self._dense_obs()

    def step(self, action):
        a = torch.as_tensor(np.asarray(action)).reshape(self.num_envs, self.S, 7).to(torch.uint8)
        self.step_compact(a)
        infos = [{} for _ in range(self.num_envs)]
        return (self._dense_obs(), self._rew.numpy().copy(), self._done.numpy().astype(bool),
                infos)

    def get_action_mask(self):
        out = np.zeros((self.num_envs, self.S, 78), dtype=np.uint8)
        self._env.dense_mask(out.ctypes.data)
        return out

    def _dense_obs(self):
        out = np.zeros((self.num_envs, self.height, self.width, 27), dtype=np.float32)
        self._env.dense_obs(out.ctypes.data)
        return out

    def render(self, mode: str = "ansi"):
        """Text render of env 0 (the reference's Java window is not available)."""
        o = self._obs[0].numpy().view(np.uint32)
        chars = {1: "$", 2: "B", 3: "K", 4: "w", 5: "l", 6: "h", 7: "r"}
        rows = []
        for y in range(self.height):
            row = ""
            for x in range(self.width):
                b = int(o[y * self.width + x])
                t = next((k for k in range(8) if b >> (13 + k) & 1), 0)
                own = next((k for k in range(3) if b >> (10 + k) & 1), 0)
                ch = chars.get(t, ".")
                row += ch.upper() if own == 1 else ch
            rows.append(row)
        s = "\n".join(rows)
        if mode == "human":
            print(s)
        return s

    def close(self):
        self._closed = True


def create_env(size: int, n_envs: int, max_steps: int, seed: int = 0, opponents=None,
               reward_weight=None, env_index_base: int = 0, env: str = "synthetic"):
    """reference libs/utils.py:59-76 create_env(size, n_envs, max_steps)."""
    if env == "microrts":
        from .microrts import create_microrts_env

        return create_microrts_env(size, n_envs, max_steps, opponents, reward_weight)
    return SyntheticGridVecEnv(num_bot_envs=n_envs, max_steps=max_steps, ai2s=opponents,
                               map_paths=[f"maps/{size}x{size}/basesWorkers{size}x{size}.xml"],
                               reward_weight=reward_weight, size=size, seed=seed,
                               env_index_base=env_index_base)
