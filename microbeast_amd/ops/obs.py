"""Observation formats.

The simulator emits one uint32 per cell whose bit p is plane p of the
gym-microRTS one-hot observation (27 planes: hp 5, resources 5, owner 3,
type 8, current action 6). The reference shipped (n, s, s, 27) float32
(env_packer.py:8-10; 27 KB per 16x16 frame) — the compact form is 1 KB.
"""
from __future__ import annotations

import torch

PLANES = 27


def bits_to_planes(obs_bits: torch.Tensor, h: int, w: int, dtype=torch.float32,
                   planes: int = PLANES) -> torch.Tensor:
    """int32 [N, h*w] -> [N, planes, h, w] (NCHW) in ``dtype``."""
    n = obs_bits.shape[0]
    sh = torch.arange(planes, device=obs_bits.device, dtype=torch.int32).view(1, planes, 1)
    x = (obs_bits.view(n, 1, h * w) >> sh) & 1
    return x.to(dtype).view(n, planes, h, w)


def bits_to_dense(obs_bits: torch.Tensor, h: int, w: int, planes: int = PLANES) -> torch.Tensor:
    """int32 [N, h*w] -> float32 [N, h, w, planes] (reference layout)."""
    return bits_to_planes(obs_bits, h, w, torch.float32, planes).permute(0, 2, 3, 1).contiguous()


def dense_to_bits(obs: torch.Tensor) -> torch.Tensor:
    """float [N, h, w, planes] one-hot -> int32 [N, h*w]."""
    n, h, w, p = obs.shape
    wts = torch.ones(p, dtype=torch.int64, device=obs.device) << torch.arange(p, device=obs.device)
    v = ((obs.reshape(n, h * w, p) > 0.5).to(torch.int64) * wts).sum(-1)
    return v.to(torch.int32)
