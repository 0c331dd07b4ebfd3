"""CSV metrics — the reference's two streams, single-writer, correct dtypes.

* ``{exp}.csv``: ``Return,steps`` (+ env_index, winner, opponent: league snapshot id of a
  self-play episode, or -1 - bot id) — one row per finished
  episode (reference microbeast.py:130-133, env_packer.py:66-75, where every
  actor process appended to the file concurrently and the header had one
  column fewer than the rows).
* ``{exp}Losses.csv``: ``update,pg_loss,value_loss,entropy_loss,total_loss,
  update time`` (reference microbeast.py:135-139, 233-239) + trailing columns
  frames, fps, wait_s, learn_s, mean_rho and the GPU phase split of the update
  (fwd_ms, bwd_ms, allreduce_ms, optim_ms, publish_ms: HIP-event times read one
  update late, so logging them never synchronises the host with the GPU) and
  policy_lag (learner updates between the rollout's behaviour weights and the
  update that consumed it).

Only rank 0 writes (DP); rows are flushed per write so a killed run keeps
its log.
"""
from __future__ import annotations

import csv
import os

EPISODE_HEADER = ["Return", "steps", "env_index", "winner", "opponent"]
PHASES = ("fwd", "bwd", "allreduce", "optim", "publish")
LOSS_HEADER = ["update", "pg_loss", "value_loss", "entropy_loss", "total_loss", "update time",
               "frames", "fps", "wait_s", "learn_s", "mean_rho"] + [f"{p}_ms" for p in PHASES] + [
               "policy_lag"]


class PhaseTimer:
    """GPU-side phase split of a learner update with HIP events, never blocking the host.

    ``start()`` / ``mark(name)`` record events on the current stream; ``read()`` returns
    {name: ms since the previous mark} of the most recent update whose events have
    COMPLETED (``query()``, not ``synchronize()``), i.e. typically the previous update.
    Double-buffered, so recording update k never overwrites events of k-1 still in flight.
    (Reference: only wall-clock per update, microbeast.py:223-231)
    """

    def __init__(self, enabled: bool = True):
        import torch

        self.enabled = enabled and torch.cuda.is_available()
        self._sets = [[], []]
        self._cur = 0
        self._last: dict = {}

    def start(self):
        if not self.enabled:
            return
        import torch

        self._cur ^= 1
        self._sets[self._cur] = [("start", torch.cuda.Event(enable_timing=True))]
        self._sets[self._cur][0][1].record()

    def mark(self, name: str):
        if not self.enabled or not self._sets[self._cur]:
            return
        import torch

        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._sets[self._cur].append((name, ev))

    def read(self) -> dict:
        if not self.enabled:
            return {}
        for idx in (self._cur, self._cur ^ 1):
            evs = self._sets[idx]
            if len(evs) > 1 and evs[-1][1].query():
                self._last = {n: evs[i - 1][1].elapsed_time(e) for i, (n, e) in enumerate(evs)
                              if i > 0}
                break
        return dict(self._last)


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
               mean_rho: float, phase_ms: dict | None = None, policy_lag: float = -1) -> None:
        if not self.enabled:
            return
        ph = phase_ms or {}
        self._lossw.writerow([update, pg, value, entropy, total, update_time, frames,
                              round(fps, 2), round(wait_s, 6), round(learn_s, 6), mean_rho]
                             + [round(ph[p], 4) if p in ph else "" for p in PHASES]
                             + [policy_lag])
        self._loss.flush()

    def close(self):
        for f in (self._ep, self._loss):
            if f is not None:
                f.close()


def read_episodes(path: str):
    with open(path) as f:
        rows = list(csv.reader(f))
    return rows[0], [[float(x) for x in r] for r in rows[1:] if r]
