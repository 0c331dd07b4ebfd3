"""V-trace targets + IMPALA losses + the loss gradients, fused.

Reference: libs/utils.py:277-329 (``PPO_learn``). Differences on purpose:
the policy-gradient sign is the correct ``-mean(logp * adv)``
and inputs are properly time-major (§8 D2).

Device tensors run the HIP kernel (``vtrace.hip``): one lane per trajectory,
reverse scan in registers, gradients written directly. CPU tensors run the
same recurrence with torch ops (also the test oracle).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import _native as N


@dataclass
class VTraceOut:
    g_logp: torch.Tensor   # [T, B] dL/dlogp
    g_value: torch.Tensor  # [T+1, B] dL/dV (row T = 0: bootstrap has no gradient)
    g_ent: float           # dL/dentropy per frame (constant)
    losses: torch.Tensor   # [5] pg, value, entropy, total, mean rho
    vs: torch.Tensor | None = None
    adv: torch.Tensor | None = None


def vtrace_torch(logp_new, logp_old, values, reward, done, entropy=None, gamma=0.99,
                 rho_bar=1.0, c_bar=1.0, pg_rho_bar=1.0, baseline_cost=0.5, entropy_cost=0.01,
                 reward_clip=0.0) -> VTraceOut:
    T, B = logp_new.shape
    lpn = logp_new.detach().float()
    ratio = torch.exp(lpn - logp_old.float())
    rho = ratio.clamp(max=rho_bar)
    cs = ratio.clamp(max=c_bar)
    r = reward.float()
    if reward_clip > 0:
        r = r.clamp(-reward_clip, reward_clip)
    disc = (~done.bool()).float() * gamma
    v = values.detach().float()
    v_t, v_tp1 = v[:T], v[1:T + 1]
    deltas = rho * (r + disc * v_tp1 - v_t)
    acc = torch.zeros(B, dtype=torch.float32, device=lpn.device)
    vs_minus_v = torch.empty_like(deltas)
    for t in range(T - 1, -1, -1):
        acc = deltas[t] + disc[t] * cs[t] * acc
        vs_minus_v[t] = acc
    vs = vs_minus_v + v_t
    vs_tp1 = torch.cat([vs[1:], v[T:T + 1]], 0)
    adv = ratio.clamp(max=pg_rho_bar) * (r + disc * vs_tp1 - v_t)
    M = float(T * B)
    g_logp = -adv / M
    g_value = torch.zeros_like(v)
    g_value[:T] = 2.0 * baseline_cost * (v_t - vs) / M
    pg = -(lpn * adv).sum() / M
    vl = baseline_cost * ((vs - v_t) ** 2).sum() / M
    ent = entropy.detach().float().sum() / M if entropy is not None else torch.zeros((), device=lpn.device)
    losses = torch.stack([pg, vl, ent, pg + vl - entropy_cost * ent, rho.mean()])
    return VTraceOut(g_logp, g_value, -entropy_cost / M, losses, vs, adv)


class VTraceWorkspace:
    """Pre-allocated device buffers so the learner step never allocates."""

    def __init__(self):
        self._bufs = {}

    def get(self, name, shape, device):
        t = self._bufs.get(name)
        if t is None or t.shape != torch.Size(shape) or t.device != device:
            t = torch.empty(shape, dtype=torch.float32, device=device)
            self._bufs[name] = t
        return t


def vtrace(logp_new, logp_old, values, reward, done, entropy=None, gamma=0.99, rho_bar=1.0,
           c_bar=1.0, pg_rho_bar=1.0, baseline_cost=0.5, entropy_cost=0.01, reward_clip=0.0,
           want_targets=False, ws: VTraceWorkspace | None = None) -> VTraceOut:
    """logp_new/logp_old/reward/done/entropy: [T, B]; values: [T+1, B]."""
    if not logp_new.is_cuda:
        return vtrace_torch(logp_new, logp_old, values, reward, done, entropy, gamma, rho_bar,
                            c_bar, pg_rho_bar, baseline_cost, entropy_cost, reward_clip)
    T, B = logp_new.shape
    dev = logp_new.device
    ws = ws or VTraceWorkspace()
    g_logp = ws.get("g_logp", (T, B), dev)
    g_value = ws.get("g_value", (T + 1, B), dev)
    partials = ws.get("partials", (((B + 255) // 256) * 4,), dev)
    losses = ws.get("losses", (5,), dev)
    vs = ws.get("vs", (T, B), dev) if want_targets else None
    adv = ws.get("adv", (T, B), dev) if want_targets else None
    c = lambda x: x.contiguous()  # noqa: E731
    lpn, lpo, val, rew = c(logp_new.detach().float()), c(logp_old.float()), c(values.detach().float()), c(reward.float())
    dn = c(done.to(torch.uint8))
    ent = c(entropy.detach().float()) if entropy is not None else None
    N.check(N.kernels().mbk_vtrace(
        lpn.data_ptr(), lpo.data_ptr(), val.data_ptr(), rew.data_ptr(), dn.data_ptr(),
        N.ptr(ent), T, B, gamma, rho_bar, c_bar, pg_rho_bar, baseline_cost, entropy_cost,
        reward_clip, N.ptr(vs), N.ptr(adv), g_logp.data_ptr(), g_value.data_ptr(),
        partials.data_ptr(), losses.data_ptr(), N.stream_ptr()), "vtrace")
    return VTraceOut(g_logp, g_value, -entropy_cost / float(T * B), losses, vs, adv)
