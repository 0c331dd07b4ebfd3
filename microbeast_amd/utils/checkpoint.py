"""Checkpoint / resume (the reference has none: SURVEY §5.4).

Format (``torch.save`` dict, loadable with ``weights_only=True``):

* ``model_state_dict`` — keys follow the reference ``Agent`` module names
  exactly (``network.{0,1,2}.conv.*``, ``network.{i}.res_block{0,1}.conv{0,1}.*``,
  ``network.5.*``, ``actor.*``, ``critic.*``), so a reference state_dict loads
  into our model and vice versa;
* ``optimizer_state_dict`` — flat Adam moments + step;
* ``step`` (env frames), ``n_update``, ``flags`` (plain dict), ``rng_state``,
  ``format``.

Rank 0 writes atomically (temp file + rename) so a crash never leaves a
truncated checkpoint.
"""
from __future__ import annotations

import dataclasses
import os

import torch

FORMAT = "microbeast_amd/1"


def save_checkpoint(path: str, model: torch.nn.Module, optimizer=None, step: int = 0,
                    n_update: int = 0, flags=None, extra: dict | None = None) -> str:
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    opt = None
    if optimizer is not None:
        o = optimizer.state_dict()
        opt = {k: (v.detach().cpu().clone() if torch.is_tensor(v) else v) for k, v in o.items()}
        if "betas" in opt:
            opt["betas"] = list(opt["betas"])
    fl = dataclasses.asdict(flags) if dataclasses.is_dataclass(flags) else (flags or {})
    ck = {"format": FORMAT, "model_state_dict": sd, "optimizer_state_dict": opt,
          "step": int(step), "n_update": int(n_update), "flags": fl,
          "rng_state": torch.get_rng_state()}
    if extra:
        ck.update(extra)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, map_location="cpu") -> dict:
    ck = torch.load(path, map_location=map_location, weights_only=True)
    if "model_state_dict" not in ck:
        # a bare reference-style state_dict
        ck = {"format": "state_dict", "model_state_dict": ck, "optimizer_state_dict": None,
              "step": 0, "n_update": 0, "flags": {}}
    return ck


def restore(ck: dict, model: torch.nn.Module, optimizer=None) -> tuple[int, int]:
    model.load_state_dict(ck["model_state_dict"])
    if optimizer is not None and ck.get("optimizer_state_dict"):
        optimizer.load_state_dict(ck["optimizer_state_dict"])
    if "rng_state" in ck and ck["rng_state"] is not None:
        torch.set_rng_state(ck["rng_state"])
    return int(ck.get("step", 0)), int(ck.get("n_update", 0))


def league_shard_path(path: str, rank: int) -> str:
    """Per-rank league state next to the main checkpoint: every DP rank plays (and matches
    opponents from) its own league, so each one's snapshots and PFSP results are saved."""
    return f"{path}.league{rank}"


def save_league_shard(path: str, rank: int, league_state: dict, n_update: int = -1) -> str:
    p = league_shard_path(path, rank)
    d = os.path.dirname(os.path.abspath(p))
    os.makedirs(d, exist_ok=True)
    st = {k: (v.detach().cpu().clone() if torch.is_tensor(v) else v)
          for k, v in league_state.items()}
    if isinstance(st.get("snaps"), dict):
        st["snaps"] = {k: v.detach().cpu().clone() for k, v in st["snaps"].items()}
    tmp = p + ".tmp"
    torch.save({"format": FORMAT, "rank": int(rank), "n_update": int(n_update), "league": st},
               tmp)
    os.replace(tmp, p)
    return p


def load_league_shard(path: str, rank: int, n_update: int | None = None) -> dict | None:
    """The rank's league shard, or None when there is none or (``n_update`` given) when it
    was written at a different update than the main checkpoint: a shard left by an earlier DP
    run must not override the newer league a later single-rank checkpoint holds."""
    p = league_shard_path(path, rank)
    if not os.path.exists(p):
        return None
    d = torch.load(p, map_location="cpu", weights_only=True)
    if n_update is not None and int(d.get("n_update", -1)) != int(n_update):
        return None
    return d.get("league")
