"""Flat parameter storage + fused Adam.

All parameters of a module become views of ONE contiguous fp32 buffer, and
their ``.grad`` views of ONE contiguous grad buffer. That makes the
optimizer one kernel launch (reference: torch.optim.Adam over per-tensor
lists, microbeast.py:200), the DP all-reduce a few large bucketed
collectives over contiguous slices (parallel/dist.py), checkpoint/publish a
single memcpy, and the inference-weight publish one D2D copy.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import _native as N

_ALIGN = 64  # elements: every parameter starts 256-B aligned


class FlatParams:
    def __init__(self, module: nn.Module, device: torch.device | str | None = None):
        self.module = module
        params = [p for p in module.parameters()]
        dev = torch.device(device) if device is not None else params[0].device
        offs, off = [], 0
        for p in params:
            offs.append(off)
            off += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.slices = []
        names = {id(p): n for n, p in module.named_parameters()}
        for p, o in zip(params, offs):
            n = p.numel()
            view = self.data[o:o + n].view_as(p)
            view.copy_(p.data.to(dev))
            p.data = view
            p.grad = self.grad[o:o + n].view_as(p)
            self.slices.append((names.get(id(p), "?"), o, n, tuple(p.shape)))
        self.params = params

    def zero_grad(self):
        self.grad.zero_()
        # autograd may have replaced a .grad (e.g. after set_to_none elsewhere): re-bind views
        for p, (_, o, n, _) in zip(self.params, self.slices):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:].data_ptr():
                p.grad = self.grad[o:o + n].view_as(p)

    def check_grad_views(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == self.grad[o:].data_ptr()
                   for p, (_, o, _, _) in zip(self.params, self.slices))


class FlatAdam:
    """Adam (torch.optim.Adam semantics) over a FlatParams buffer.

    Optional global-norm gradient clipping (``max_grad_norm`` > 0) and an
    optional bf16 shadow copy of the parameters written in the same kernel.
    """

    def __init__(self, flat: FlatParams, lr=2.5e-4, betas=(0.9, 0.999), eps=1e-5,
                 weight_decay=0.0, max_grad_norm=0.0, bf16_shadow: bool = False):
        self.flat = flat
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        dev = flat.data.device
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self.step_count = 0
        self.shadow = torch.empty(flat.numel, dtype=torch.bfloat16, device=dev) if bf16_shadow else None
        self._partials = torch.empty(1024, dtype=torch.float32, device=dev)
        self._scale = torch.ones(2, dtype=torch.float32, device=dev)
        self.last_grad_norm = None

    def state_dict(self):
        return {"m": self.m, "v": self.v, "step": self.step_count, "lr": self.lr,
                "betas": self.betas, "eps": self.eps}

    def load_state_dict(self, sd):
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.step_count = int(sd["step"])

    def step(self, grad_scale: float = 1.0):
        """grad_scale multiplies the gradient inside the update (the data-parallel 1/world
        average is folded in here instead of a separate pass over the buffer)."""
        self.step_count += 1
        b1, b2 = self.betas
        f = self.flat
        if f.data.is_cuda:
            k = N.kernels()
            st = N.stream_ptr()
            scale = None
            if self.max_grad_norm > 0:
                N.check(k.mbk_grad_clip_scale(f.grad.data_ptr(), f.numel, self.max_grad_norm,
                                              grad_scale, self._partials.data_ptr(), self._scale.data_ptr(),
                                              st), "grad_clip_scale")
                scale = self._scale.data_ptr()
                self.last_grad_norm = self._scale[1]
            N.check(k.mbk_adam(f.data.data_ptr(), f.grad.data_ptr(), self.m.data_ptr(),
                               self.v.data_ptr(), N.ptr(self.shadow), f.numel, self.lr, b1, b2,
                               self.eps, self.wd, self.step_count, scale, grad_scale, st),
                    "adam")
            return
        g = f.grad if grad_scale == 1.0 else f.grad * grad_scale
        if self.max_grad_norm > 0:
            norm = g.norm()
            self.last_grad_norm = norm
            g = g * torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0)
        if self.wd:
            g = g + self.wd * f.data
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        denom = (self.v.sqrt() / math.sqrt(bc2)).add_(self.eps)
        f.data.addcdiv_(self.m, denom, value=-self.lr / bc1)
        if self.shadow is not None:
            self.shadow.copy_(f.data)
