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
from ..ops.pixconv import Cells, PixPlan, gridnet_pbc, pbc_to_cell_major
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
        self.emulate = False      # run the grid path's torch emulation off-GPU (tests)
        # logits of the active cells only (compact rows) when acting / scoring; 0: dense
        self.sparse_logits = True
        self._grid_plan = None
        for p in self.parameters():  # grid-path kernels write gradients into flat slots
            p._mbk_direct_grad = True

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

    def direct_grad_ok(self, device) -> bool:
        """the grid path's backward writes every gradient into its flat slot"""
        return self.hip_kernels and (torch.device(device).type == "cuda" or self.emulate)

    def _use_hip(self, obs) -> bool:
        return self.hip_kernels and obs.dtype == torch.int32 and (obs.is_cuda or self.emulate)

    def _plan(self, device) -> PixPlan:
        if self._grid_plan is None or self._grid_plan.device != torch.device(device):
            convs = [self.encoder[i] for i in (0, 3, 6, 9)]
            convts = [self.actor[i] for i in (0, 2, 4, 6)]
            self._grid_plan = PixPlan(convs, convts, self.critic[1], self.critic[3], self.ph,
                                      self.pw, (self.h, self.w), device)
        return self._grid_plan

    def policy_value_pbc(self, obs, n_logits=None, cells=None):
        """The whole network on the pixel-major layout (ops/pixconv.py, pixconv.hip): per
        output-pixel MFMA GEMMs with no padded halo, no ATen kernel. relu(maxpool(conv)) is
        computed as maxpool(relu-fused conv): identical values. Returns (logits [h*w][n_s][96]
        bf16 pixel-major -- what the masked-cell kernels read as they are --, value fp32 [n]);
        the decoder runs on the first n_logits observations only. With ``cells`` the logits
        are the compact rows of those active cells (ops/pixconv.py Cells)."""
        n = obs.numel() // (self.h * self.w)
        return gridnet_pbc(self._plan(obs.device), obs.reshape(n, self.h * self.w),
                           self.h, self.w, self.ph, self.pw, n_logits, cells)

    def policy_value(self, obs):
        if self._use_hip(obs):
            lg, v = self.policy_value_pbc(obs)
            return pbc_to_cell_major(lg), v
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
    def act(self, obs, mask_bits, rng_state=None, generator=None, action_out=None,
            cell_logp=None, logp_out=None):
        if self._use_hip(obs):
            n = obs.numel() // (self.h * self.w)
            if self.sparse_logits:
                cells = Cells(mask_bits, n, self.h * self.w)
                zc, value = self.policy_value_pbc(obs, cells=cells)
                action, logp = cell_head.sample_rows(zc, cells, mask_bits, rng_state, generator,
                                                     action_out, cell_logp, logp_out)
                return action, logp, value
            lg, value = self.policy_value_pbc(obs)
            action, logp = cell_head.sample_pbc(lg, mask_bits, rng_state, generator, action_out,
                                                cell_logp, logp_out)
            return action, logp, value
        logits, value = self.policy_value(obs)
        action, logp = cell_head.sample(logits, mask_bits, rng_state, generator)
        return action, logp, value

    def evaluate(self, obs, mask_bits, action, n_score: int | None = None):
        if self._use_hip(obs):  # logits of the scored rows only
            if self.sparse_logits:
                ns = obs.numel() // (self.h * self.w) if n_score is None else n_score
                cells = Cells(mask_bits.reshape(ns, -1, 3).contiguous(), ns, self.h * self.w)
                zc, value = self.policy_value_pbc(obs, n_score, cells)
                logp, ent = cell_head.score_rows(zc, cells, mask_bits, action)
                return logp, ent, value
            lg, value = self.policy_value_pbc(obs, n_score)
            logp, ent = cell_head.score_pbc(lg, mask_bits, action)
            return logp, ent, value
        logits, value = self.policy_value(obs)
        if n_score is not None:
            logits = logits[:n_score]
        logp, ent = cell_head.score(logits, mask_bits, action)
        return logp, ent, value
