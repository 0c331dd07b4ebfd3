"""``--test`` mode: evaluate a checkpoint (the reference's ``test()`` is a stub
that prints "Testing...", microbeast.py:267-268)."""
from __future__ import annotations

import csv
import os

import torch

from .config import Flags
from .envs.synthetic import create_env
from .models.factory import make_model
from .utils.checkpoint import load_checkpoint


def evaluate(flags: Flags, checkpoint: str | None = None, greedy: bool = False) -> dict:
    dev = torch.device("cuda" if (flags.device != "cpu" and torch.cuda.is_available()) else "cpu")
    path = checkpoint or flags.checkpoint or os.path.join(flags.savedir, f"{flags.exp_name}.ckpt")
    model = make_model(flags, dev)
    if os.path.exists(path):
        ck = load_checkpoint(path)
        model.load_state_dict(ck["model_state_dict"])
        src = path
    elif flags.allow_random_init:
        src = "random-init (no checkpoint found, --allow_random_init)"
    else:  # an evaluation of untrained weights must not pass for a checkpoint's result
        raise FileNotFoundError(
            f"--test: no checkpoint at {path!r}; train first, pass --checkpoint PATH, or "
            f"--allow_random_init to evaluate random-init weights")
    model.eval()
    n = flags.n_envs
    env = create_env(flags.env_size, n, flags.max_episode_steps, seed=flags.seed + 777,
                     opponents=flags.opponent_list(), reward_weight=flags.reward_weights(),
                     env=flags.env)
    S = flags.env_size ** 2
    obs = torch.zeros(n, S, dtype=torch.int32)
    mask = torch.zeros(n, S, 3, dtype=torch.int32)
    env.reset_compact(obs, mask)
    rng = torch.tensor([flags.seed * 31 + 5, 0], dtype=torch.int64, device=dev)
    gen = torch.Generator().manual_seed(flags.seed)
    episodes = []
    steps = 0
    while len(episodes) < flags.eval_episodes and steps < 100 * flags.max_episode_steps:
        with torch.no_grad():
            o, m = obs.to(dev), mask.to(dev)
            if greedy:
                from .ops import cell_head
                logits, _ = model.policy_value(o)
                a = cell_head.greedy(logits, m)
            else:
                a, _, _ = model.act(o, m, rng_state=rng if dev.type == "cuda" else None,
                                    generator=gen)
        env.step_compact(a.cpu())
        episodes.extend(env.drain_episodes())
        steps += 1
    episodes = episodes[:flags.eval_episodes]
    out_path = os.path.join(flags.savedir, f"{flags.exp_name}_eval.csv")
    os.makedirs(flags.savedir or ".", exist_ok=True)
    with open(out_path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Return", "steps", "env_index", "winner"])
        for r in episodes:
            w.writerow([float(r[0]), int(r[1]), int(r[2]), int(r[3])])
    rets = [float(r[0]) for r in episodes]
    res = {"checkpoint": src, "episodes": len(episodes),
           "mean_return": sum(rets) / max(len(rets), 1),
           "win_rate": sum(1 for r in episodes if r[3] == 0) / max(len(episodes), 1),
           "csv": out_path}
    print(f"Testing... {res}", flush=True)
    return res
