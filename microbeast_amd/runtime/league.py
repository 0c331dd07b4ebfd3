"""Self-play league: a pool of past policy snapshots with PFSP matchmaking.

BASELINE config 5 ("16x16 self-play league"). The reference creates its envs with
``num_selfplay_envs=0`` (libs/utils.py:65) and only ever plays scripted bots; this
adds the standard league loop (AlphaStar-style prioritized fictitious self-play):

* every ``snapshot_every`` learner updates the current weights are frozen into the
  pool (an HBM copy of the flat fp32 parameter buffer: 21 MB at 16x16, so even a
  few hundred snapshots are a rounding error in 288 GB);
* each update an opponent is drawn with probability proportional to
  ``(1 - win_rate)^p`` (hard-opponent weighting) mixed with ``eps`` uniform, and
  swapped into the GPU engine's opponent policy through its event-ordered publish
  channel (``GpuEngine.publish_opponent``);
* finished self-play episodes come back tagged with the opponent snapshot id that
  was playing, and update that snapshot's win rate (draws count half).
"""
from __future__ import annotations

import random

import torch


class League:
    def __init__(self, capacity: int = 64, snapshot_every: int = 20, pfsp_power: float = 2.0,
                 eps: float = 0.1, seed: int = 0):
        self.capacity = capacity
        self.snapshot_every = max(1, snapshot_every)
        self.p = pfsp_power
        self.eps = eps
        self.rng = random.Random(seed)
        self.snaps: dict[int, torch.Tensor] = {}
        self.games: dict[int, float] = {}
        self.wins: dict[int, float] = {}
        self.next_id = 0
        self.current = -1

    def __len__(self):
        return len(self.snaps)

    # ------------------------------------------------------------ pool
    def add_snapshot(self, flat: torch.Tensor) -> int:
        """Freeze a copy of the flat parameter buffer (same device) into the pool."""
        sid = self.next_id
        self.next_id += 1
        self.snaps[sid] = flat.detach().clone()
        self.games.setdefault(sid, 0.0)
        self.wins.setdefault(sid, 0.0)
        while len(self.snaps) > self.capacity:
            # evict the snapshot the learner beats most reliably (never the newest)
            old = max((k for k in self.snaps if k != sid), key=self.win_rate)
            del self.snaps[old]
        return sid

    def maybe_snapshot(self, update: int, flat: torch.Tensor) -> int | None:
        if update % self.snapshot_every == 0 or not self.snaps:
            return self.add_snapshot(flat)
        return None

    # ------------------------------------------------------------ results
    def win_rate(self, sid: int) -> float:
        """Learner's win rate against snapshot ``sid`` (Beta(1,1) prior)."""
        return (self.wins.get(sid, 0.0) + 1.0) / (self.games.get(sid, 0.0) + 2.0)

    def record(self, episodes) -> None:
        """episodes: (return, length, env_index, winner, opponent) tuples."""
        for ep in episodes:
            if len(ep) < 5 or ep[4] < 0:
                continue  # scripted-bot episode
            sid, winner = int(ep[4]), int(ep[3])
            self.games[sid] = self.games.get(sid, 0.0) + 1.0
            self.wins[sid] = self.wins.get(sid, 0.0) + (1.0 if winner == 0 else
                                                        0.5 if winner < 0 else 0.0)

    # ------------------------------------------------------------ matchmaking
    def weights(self) -> dict[int, float]:
        ids = list(self.snaps)
        hard = {k: (1.0 - self.win_rate(k)) ** self.p for k in ids}
        tot = sum(hard.values()) or 1.0
        n = len(ids)
        return {k: (1 - self.eps) * hard[k] / tot + self.eps / n for k in ids}

    def sample(self) -> int:
        w = self.weights()
        ids = list(w)
        return self.rng.choices(ids, weights=[w[k] for k in ids], k=1)[0]

    def snapshot(self, sid: int) -> torch.Tensor:
        return self.snaps[sid]

    def summary(self) -> dict:
        return {"size": len(self.snaps), "current": self.current,
                "win_rate": {k: round(self.win_rate(k), 3) for k in self.snaps},
                "games": {k: int(self.games.get(k, 0)) for k in self.snaps}}

    # ------------------------------------------------------------ checkpoint
    def state_dict(self, with_snapshots: bool = True) -> dict:
        d = {"next_id": self.next_id, "games": dict(self.games), "wins": dict(self.wins),
             "current": self.current}
        if with_snapshots:
            d["snaps"] = {k: v.cpu() for k, v in self.snaps.items()}
        return d

    def load_state_dict(self, d: dict, device=None) -> None:
        self.next_id = int(d["next_id"])
        self.games = {int(k): float(v) for k, v in d["games"].items()}
        self.wins = {int(k): float(v) for k, v in d["wins"].items()}
        self.current = int(d.get("current", -1))
        if "snaps" in d:
            self.snaps = {int(k): v.to(device) for k, v in d["snaps"].items()}
