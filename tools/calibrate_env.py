#!/usr/bin/env python
"""Calibrate the native microRTS stand-in against the reference's own training logs.

The reference's two logged runs (experiments/24_dic, experiments/5_ener) never learned (SURVEY
§8 D1: the optimizer never touched the acting model), so they record its INITIAL policy: the
actor head has orthogonal gain 0 (reference model.py:136), i.e. every component is uniform over
its legal choices, against the bot mix 3 x coacAI, randomBiasedAI, lightRushAI, workerRushAI
(reference libs/utils.py:69-72), reward weights [10, 1, 1, 0.2, 1, 4] (libs/utils.py:74), most
likely on 8x8. This tool plays that policy in the stand-in (C++ simulator, same reward weights
and bot mix) and prints the statistics the logs give:

  mean episode length (logs: ~300 steps), mean return (~ -2), share of episodes with return
  >= 10 (~3.5 %: wins), and the active-cell fraction the sparse head sees.

  python tools/calibrate_env.py --size 8 --envs 240 --steps 4000 [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SEG = [0, 6, 10, 14, 18, 22, 29, 78]
REFERENCE = {"mean_len": 300.0, "mean_return": -2.0, "win_share": 0.035,
             "source": "experiments/5_ener/5_enero.csv, experiments/24_dic/24_dic.csv "
                       "(SURVEY §6.1: length ~300, return -2.26..-1.85, return>=10 3.4-4.2 %)"}


def uniform_legal(mask_bits: np.ndarray, rng: np.random.Generator) -> np.ndarray:
    """One uniform draw per component among the legal choices (Gumbel-max over the mask)."""
    n, S, _ = mask_bits.shape
    w = mask_bits.view(np.uint32)
    bits = ((w[..., :, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(n, S, 96)[..., :78]
    g = rng.gumbel(size=bits.shape).astype(np.float32)
    score = np.where(bits > 0, g, -np.inf)
    a = np.zeros((n, S, 7), np.uint8)
    for k in range(7):
        seg = score[..., SEG[k]:SEG[k + 1]]
        idx = np.argmax(seg, axis=-1)
        idx[~np.isfinite(seg.max(-1))] = 0
        a[..., k] = idx
    return a


def run(size: int, envs: int, steps: int, seed: int, max_steps: int, bots=None) -> dict:
    import torch

    from microbeast_amd import _native as N
    from microbeast_amd.runtime.gpu_actors import BOT_IDS, DEFAULT_BOTS

    rt = N.runtime()
    S = size * size
    ids = [BOT_IDS[b] for b in (bots or DEFAULT_BOTS)]
    env = rt.VecEnv(size, envs, max_steps, seed, ids)
    obs = torch.zeros(envs, S, dtype=torch.int32)
    mask = torch.zeros(envs, S, 3, dtype=torch.int32)
    rew = torch.zeros(envs)
    done = torch.zeros(envs, dtype=torch.uint8)
    env.reset(obs.data_ptr(), mask.data_ptr())
    rng = np.random.default_rng(seed)
    active = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        m = mask.numpy()
        active += float((m != 0).any(-1).mean())
        a = torch.from_numpy(uniform_legal(m, rng))
        env.step(a.data_ptr(), obs.data_ptr(), mask.data_ptr(), rew.data_ptr(), done.data_ptr())
    eps = env.drain_episodes()
    wall = time.perf_counter() - t0
    ret = np.array([e[0] for e in eps], np.float64)
    ln = np.array([e[1] for e in eps], np.float64)
    win = np.array([e[3] for e in eps]) if eps and len(eps[0]) > 3 else np.zeros(0)
    per_bot = {}
    for e in eps:
        b = (bots or DEFAULT_BOTS)[int(e[2]) % len(bots or DEFAULT_BOTS)]
        d = per_bot.setdefault(b, [0, 0.0, 0.0])
        d[0] += 1
        d[1] += e[1]
        d[2] += float(e[0] >= 10)
    return {
        "size": size, "envs": envs, "steps": steps, "episodes": len(eps),
        "mean_len": float(ln.mean()) if len(ln) else None,
        "median_len": float(np.median(ln)) if len(ln) else None,
        "mean_return": float(ret.mean()) if len(ret) else None,
        "win_share_return_ge_10": float((ret >= 10).mean()) if len(ret) else None,
        "win_share_engine": float((win == 0).mean()) if len(win) else None,
        "timeout_share": float((ln >= max_steps).mean()) if len(ln) else None,
        "active_cell_fraction": active / steps,
        "per_bot": {b: {"episodes": v[0], "mean_len": round(v[1] / v[0], 1),
                        "win_share": round(v[2] / v[0], 4)} for b, v in per_bot.items()},
        "reference": REFERENCE, "wall_s": round(wall, 1),
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=8)
    p.add_argument("--envs", type=int, default=240)
    p.add_argument("--steps", type=int, default=4000)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--max_steps", type=int, default=2000)
    p.add_argument("--json", type=str, default="")
    a = p.parse_args()
    out = run(a.size, a.envs, a.steps, a.seed, a.max_steps)
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
