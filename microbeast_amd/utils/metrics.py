"""CSV metrics — the reference's two streams, single-writer, correct dtypes.

* ``{exp}.csv``: ``Return,steps`` (+ env_index, winner, opponent: league snapshot id of a
  self-play episode, or -1 - bot id) — one row per finished
  episode (reference microbeast.py:130-133, env_packer.py:66-75, where every
  actor process appended to the file concurrently and the header had one
  column fewer than the rows).
* ``{exp}Losses.csv``: ``update,pg_loss,value_loss,entropy_loss,total_loss,
  update time`` (reference microbeast.py:135-139, 233-239) + trailing columns
  frames, fps, wait_s, learn_s, mean_rho.

Only rank 0 writes (DP); rows are flushed per write so a killed run keeps
its log.
"""
from __future__ import annotations

import csv
import os

EPISODE_HEADER = ["Return", "steps", "env_index", "winner", "opponent"]
LOSS_HEADER = ["update", "pg_loss", "value_loss", "entropy_loss", "total_loss", "update time",
               "frames", "fps", "wait_s", "learn_s", "mean_rho"]


class CsvLogger:
    def __init__(self, savedir: str, exp_name: str, enabled: bool = True, append: bool = False):
        self.enabled = enabled
        self.ep_path = os.path.join(savedir, f"{exp_name}.csv")
        self.loss_path = os.path.join(savedir, f"{exp_name}Losses.csv")
        self._ep = self._loss = None
        if not enabled:
            return
        os.makedirs(savedir or ".", exist_ok=True)
        mode = "a" if append else "w"
        new_ep = not (append and os.path.exists(self.ep_path))
        new_loss = not (append and os.path.exists(self.loss_path))
        self._ep = open(self.ep_path, mode, newline="")
        self._loss = open(self.loss_path, mode, newline="")
        self._epw = csv.writer(self._ep)
        self._lossw = csv.writer(self._loss)
        if new_ep:
            self._epw.writerow(EPISODE_HEADER)
        if new_loss:
            self._lossw.writerow(LOSS_HEADER)
        self._ep.flush()
        self._loss.flush()
        self.n_episodes = 0

    def episodes(self, recs) -> None:
        if not self.enabled or not recs:
            return
        for r in recs:
            ret, length, env_idx, winner = r[:4]
            opp = r[4] if len(r) > 4 else -1
            self._epw.writerow([float(ret), int(length), int(env_idx), int(winner), int(opp)])
        self.n_episodes += len(recs)
        self._ep.flush()

    def losses(self, update: int, pg: float, value: float, entropy: float, total: float,
               update_time: float, frames: int, fps: float, wait_s: float, learn_s: float,
               mean_rho: float) -> None:
        if not self.enabled:
            return
        self._lossw.writerow([update, pg, value, entropy, total, update_time, frames,
                              round(fps, 2), round(wait_s, 6), round(learn_s, 6), mean_rho])
        self._loss.flush()

    def close(self):
        for f in (self._ep, self._loss):
            if f is not None:
                f.close()


def read_episodes(path: str):
    with open(path) as f:
        rows = list(csv.reader(f))
    return rows[0], [[float(x) for x in r] for r in rows[1:] if r]
