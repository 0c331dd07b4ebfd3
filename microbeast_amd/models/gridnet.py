"""GridNet encoder-decoder agent (BASELINE config 2: "10x10 GridNet CNN").

The reference only ships the flat IMPALA head (model.py); GridNet is the
standard gym-microRTS architecture (Huang et al., "Gym-μRTS", 2021): a
strided conv encoder, a transposed-conv decoder that emits 78 logits for every
map cell directly (so the head has no 256 x 78*h*w matrix), and a small
critic. Its logits are cell-major like the flat head, so the same masked-cell
kernels (``ops/cell_head``) sample / score it.

Map sizes are padded up to a multiple of 16 internally (the encoder halves 4
times); logits of padding cells are dropped.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import cell_head
from ..ops.gridconv import conv3x3, conv_transpose3x3s2, maxpool3x3s2
from ..ops.linear import linear
from ..ops.obs import bits_to_planes
from .agent import layer_init


class GridNetAgent(nn.Module):
    def __init__(self, obs_space_shape=(16, 16, 27), compute_dtype=torch.bfloat16,
                 hip_kernels: bool = True):
        super().__init__()
        self.hip_kernels = hip_kernels
        h, w, c = obs_space_shape
        self.h, self.w, self.planes = h, w, c
        self.ph, self.pw = -(-h // 16) * 16, -(-w // 16) * 16
        self.encoder = nn.Sequential(
            layer_init(nn.Conv2d(c, 32, 3, padding=1)), nn.MaxPool2d(3, 2, 1), nn.ReLU(),
            layer_init(nn.Conv2d(32, 64, 3, padding=1)), nn.MaxPool2d(3, 2, 1), nn.ReLU(),
            layer_init(nn.Conv2d(64, 128, 3, padding=1)), nn.MaxPool2d(3, 2, 1), nn.ReLU(),
            layer_init(nn.Conv2d(128, 256, 3, padding=1)), nn.MaxPool2d(3, 2, 1), nn.ReLU())
        self.actor = nn.Sequential(
            layer_init(nn.ConvTranspose2d(256, 128, 3, 2, 1, 1)), nn.ReLU(),
            layer_init(nn.ConvTranspose2d(128, 64, 3, 2, 1, 1)), nn.ReLU(),
            layer_init(nn.ConvTranspose2d(64, 32, 3, 2, 1, 1)), nn.ReLU(),
            layer_init(nn.ConvTranspose2d(32, cell_head.CELL, 3, 2, 1, 1), std=0.01))
        flat = 256 * (self.ph // 16) * (self.pw // 16)
        self.critic = nn.Sequential(nn.Flatten(), layer_init(nn.Linear(flat, 128)), nn.ReLU(),
                                    layer_init(nn.Linear(128, 1), std=1))
        self.compute_dtype = compute_dtype
        self.nvec = list(cell_head.NVEC) * (h * w)

    def _planes(self, obs):
        if obs.dtype == torch.int32:
            x = bits_to_planes(obs.reshape(-1, self.h * self.w), self.h, self.w, torch.float32,
                               self.planes)
        else:
            x = obs.reshape(-1, self.h, self.w, self.planes).permute(0, 3, 1, 2).float()
        if (self.ph, self.pw) != (self.h, self.w):
            x = F.pad(x, (0, self.pw - self.w, 0, self.ph - self.h))
        return x

    def _autocast(self, t):
        return torch.autocast("cuda", dtype=self.compute_dtype,
                              enabled=t.is_cuda and self.compute_dtype != torch.float32,
                              cache_enabled=False)

    def _use_hip(self, obs) -> bool:
        return self.hip_kernels and obs.is_cuda and obs.dtype == torch.int32

    def _policy_value_hip(self, obs):
        """Every conv / transposed conv on the MFMA GEMM (ops/gridconv.py), NHWC bf16.
        relu(maxpool(conv)) is computed as maxpool(relu-fused conv): identical values."""
        n = obs.numel() // (self.h * self.w)
        bits = obs.reshape(n, self.h, self.w, 1)
        sh = torch.arange(32, device=obs.device, dtype=torch.int32)
        x = ((bits >> sh) & 1).to(torch.bfloat16)  # planes 27..31 are zero: Cin 27 -> 32
        if (self.ph, self.pw) != (self.h, self.w):
            x = F.pad(x, (0, 0, 0, self.pw - self.w, 0, self.ph - self.h))
        for i in (0, 3, 6, 9):
            conv = self.encoder[i]
            x = maxpool3x3s2(conv3x3(x, conv.weight, conv.bias, relu=True))
        z = x  # NHWC [n, ph/16, pw/16, 256]
        y = z
        for j, i in enumerate((0, 2, 4, 6)):
            ct = self.actor[i]
            last = j == 3
            y = conv_transpose3x3s2(y, ct.weight, ct.bias, relu=not last, nchw_out=last)
        logits = y[:, :, :self.h, :self.w].permute(0, 2, 3, 1).reshape(n, -1).float()
        zf = z.permute(0, 3, 1, 2).reshape(n, -1)  # the reference's NCHW flatten order
        hdn = F.relu(linear(zf, self.critic[1]))
        v = linear(hdn, self.critic[3])
        return logits, v.float().view(-1)

    def policy_value(self, obs):
        if self._use_hip(obs):
            return self._policy_value_hip(obs)
        x = self._planes(obs)
        with self._autocast(x):
            z = self.encoder(x)
            lg = self.actor(z)[:, :, :self.h, :self.w]
            v = self.critic(z)
        logits = lg.permute(0, 2, 3, 1).reshape(lg.shape[0], -1).float()
        return logits, v.float().view(-1)

    def initial_state(self, batch_size: int = 1):
        return tuple()

    @torch.no_grad()
    def act(self, obs, mask_bits, rng_state=None, generator=None):
        logits, value = self.policy_value(obs)
        action, logp = cell_head.sample(logits, mask_bits, rng_state, generator)
        return action, logp, value

    def evaluate(self, obs, mask_bits, action, n_score: int | None = None):
        logits, value = self.policy_value(obs)
        if n_score is not None:
            logits = logits[:n_score]
        logp, ent = cell_head.score(logits, mask_bits, action)
        return logp, ent, value
