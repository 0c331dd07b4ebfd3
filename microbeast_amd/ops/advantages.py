"""TD errors and (generalized) advantage estimates over [n_envs, T+1] rollouts.

The reference carries these as dead code next to V-trace (libs/utils.py:104-127
``get_deltas``, :130-163 ``get_advantages``, :78-101 ``flatten_batch_and_advantages``;
never called). They are provided here as O(T) reverse scans instead of the
reference's O(T^2) double loop:

* ``td_deltas``: delta_t = r_t + gamma * V_{t+1} * (1 - done_t) - V_t for t < T, 0 at T
  (exactly ``get_deltas``);
* ``advantages``: A_t = sum_k (gamma * lam)^(k-t) delta_k. With ``reference=True`` the
  discount runs straight through episode ends like ``get_advantages`` (lam = 1); the
  default stops the sum at ``done`` (proper GAE).
"""
from __future__ import annotations

import torch


def td_deltas(reward: torch.Tensor, value: torch.Tensor, done: torch.Tensor,
              gamma: float) -> torch.Tensor:
    """[n, T+1] -> [n, T+1] (last column 0)."""
    d = torch.zeros_like(value, dtype=torch.float32)
    nd = 1.0 - done[:, :-1].float()
    d[:, :-1] = reward[:, :-1].float() + gamma * value[:, 1:].float() * nd - value[:, :-1].float()
    return d


def advantages(reward: torch.Tensor, value: torch.Tensor, done: torch.Tensor, gamma: float,
               lam: float = 1.0, reference: bool = False) -> torch.Tensor:
    """[n, T+1] -> [n, T+1] advantage estimates (last column 0)."""
    delta = td_deltas(reward, value, done, gamma)
    out = torch.zeros_like(delta)
    acc = torch.zeros(delta.shape[0], dtype=delta.dtype, device=delta.device)
    for t in range(delta.shape[1] - 2, -1, -1):
        carry = gamma * lam * acc
        if not reference:
            carry = carry * (1.0 - done[:, t].float())
        acc = delta[:, t] + carry
        out[:, t] = acc
    return out


def flatten_batch_and_advantages(batch: dict, adv: torch.Tensor) -> tuple[dict, torch.Tensor]:
    """Flatten every [n, T+1, ...] batch entry to [1, n*(T+1), ...] (``ep_step`` to 1-D) and
    the advantages to 1-D — the reference helper's layout (libs/utils.py:78-101)."""
    out = {}
    for k, v in batch.items():
        out[k] = v.reshape(-1) if k == "ep_step" else v.reshape((1, -1) + tuple(v.shape[2:]))
    return out, adv.flatten()
