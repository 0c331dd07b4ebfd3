"""IMPALA learner step: forward -> V-trace -> backward -> all-reduce -> Adam.

Reference: ``PPO_learn`` (libs/utils.py:223-342) + the learner loop
(microbeast.py:211-248). Re-designed:

* the batch is time-major ``[T+1, B, ...]`` and stays that way (no
  reshape scrambling); row t holds obs_t/mask_t with the action
  a_t sampled there (D3 fixed);
* one model, one optimizer over a flat fp32 buffer (D1 fixed);
* the V-trace kernel returns dL/dlogp, dL/dV, dL/dH directly and backward is
  seeded with them (``autograd.backward`` on three outputs) — no scalar
  loss graph, no extra reductions;
* gradients are all-reduced in buckets overlapped with backward (DP);
* nothing syncs the host inside ``learn`` except the optional loss readout.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from .ops.copy import full
from .ops.optim import FlatAdam, FlatParams
from .ops.vtrace import VTraceWorkspace, vtrace
from .parallel.dist import DistInfo, GradAllReducer, broadcast_flat
from .utils.metrics import PhaseTimer


@dataclass
class LearnerHParams:
    lr: float = 2.5e-4          # microbeast.py:200
    adam_eps: float = 1e-5      # microbeast.py:200
    gamma: float = 0.99         # microbeast.py:118 / libs/utils.py:277
    baseline_cost: float = 0.5  # libs/utils.py:323 (0.5 * mean sq)
    entropy_cost: float = 0.01  # libs/utils.py:329
    rho_bar: float = 1.0        # libs/utils.py:293
    c_bar: float = 1.0          # libs/utils.py:294
    pg_rho_bar: float = 1.0     # libs/utils.py:316
    reward_clip: float = 0.0    # reference: none
    max_grad_norm: float = 0.0  # reference: none
    bucket_mb: float = 8.0
    allreduce_dtype: str = "fp32"  # fp32 | bf16 (gradient all-reduce payload)
    comm_rehearsal: bool = False   # world 1: stand-in collectives on a 4th stream (dist.py)


class Learner:
    def __init__(self, model: torch.nn.Module, hp: LearnerHParams, device: torch.device,
                 info: DistInfo | None = None):
        self.model = model.to(device)
        self.device = device
        self.hp = hp
        self.info = info or DistInfo()
        self.flat = FlatParams(self.model, device)
        broadcast_flat(self.flat, self.info)
        self.opt = FlatAdam(self.flat, lr=hp.lr, eps=hp.adam_eps, max_grad_norm=hp.max_grad_norm)
        self.reducer = GradAllReducer(
            self.flat, self.info, hp.bucket_mb,
            torch.bfloat16 if hp.allreduce_dtype == "bf16" else torch.float32,
            rehearse=hp.comm_rehearsal)
        self.ws = VTraceWorkspace()
        self.n_updates = 0
        self.timing = {}
        # HIP-event split fwd / bwd / allreduce(wait) / optim (+ publish marked by the
        # caller), read one update late without a host sync
        self.phases = PhaseTimer(enabled=device.type == "cuda")

    def learn(self, batch: dict, sync_timing: bool = False) -> torch.Tensor:
        """batch keys (time-major): obs [T+1,B,...], mask [T+1,B,S,3] int32,
        action [T+1,B,S,7] uint8, logp [T+1,B], reward [T+1,B], done [T+1,B].
        Returns the device tensor [5] = pg, value, entropy, total, mean rho."""
        t0 = time.perf_counter()
        self.phases.start()
        obs, mask, action = batch["obs"], batch["mask"], batch["action"]
        T1, B = batch["logp"].shape[:2]
        T = T1 - 1
        self.flat.zero_grad()
        self.reducer.start_step()
        flat_obs = obs.reshape(T1 * B, *obs.shape[2:])
        S = mask.shape[2]
        m = mask[:T].reshape(T * B, S, mask.shape[-1])
        a = action[:T].reshape(T * B, S, action.shape[-1])
        kw = {}
        ab = batch.get("abits")
        if ab is not None and getattr(self.model, "accepts_abits", False):
            # the acting step's active-cell bitmap: the head compaction skips the mask pass
            kw["abits"] = ab[:T].reshape(T * B, ab.shape[-1])
        logp, ent, value = self.model.evaluate(flat_obs, m, a, n_score=T * B, **kw)
        vt = vtrace(logp.view(T, B), batch["logp"][:T], value.view(T1, B), batch["reward"][:T],
                    batch["done"][:T], ent.view(T, B), gamma=self.hp.gamma, rho_bar=self.hp.rho_bar,
                    c_bar=self.hp.c_bar, pg_rho_bar=self.hp.pg_rho_bar,
                    baseline_cost=self.hp.baseline_cost, entropy_cost=self.hp.entropy_cost,
                    reward_clip=self.hp.reward_clip, ws=self.ws)
        self.phases.mark("fwd")
        if sync_timing and logp.is_cuda:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        torch.autograd.backward(
            [logp, value, ent], [vt.g_logp.reshape(-1), vt.g_value.reshape(-1),
                                 self._const_grad(ent, vt.g_ent)])
        if self.flat.adopt_grads() and self.info.enabled:
            raise RuntimeError("a direct-gradient parameter's gradient was not written into "
                               "its flat slot; its all-reduce bucket went out stale")
        self.phases.mark("bwd")
        self.reducer.finish()
        self.phases.mark("allreduce")
        if sync_timing and logp.is_cuda:
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        self.opt.step(grad_scale=self.reducer.grad_scale)
        self.phases.mark("optim")
        if sync_timing and logp.is_cuda:
            torch.cuda.synchronize()
        t3 = time.perf_counter()
        self.n_updates += 1
        self.timing = {"fwd_s": t1 - t0, "bwd_allreduce_s": t2 - t1, "optim_s": t3 - t2}
        return vt.losses

    def _const_grad(self, like: torch.Tensor, value: float) -> torch.Tensor:
        """constant seed gradient (entropy term), filled once per shape / value"""
        c = getattr(self, "_cg", None)
        if c is None or c[0] != (like.shape, like.device, value):
            c = ((like.shape, like.device, value), full(like.shape, value, like.dtype, like.device))
            self._cg = c
        return c[1]

    def state_dict(self):
        return {"model": self.model.state_dict(), "optim": self.opt.state_dict(),
                "n_updates": self.n_updates}

    def load_state_dict(self, sd):
        self.model.load_state_dict(sd["model"])
        self.opt.load_state_dict(sd["optim"])
        self.n_updates = int(sd.get("n_updates", 0))
