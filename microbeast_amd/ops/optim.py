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
from .copy import full, zero_, zeros

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
        self.data = zeros(off, device=dev)
        self.grad = zeros(off, device=dev)
        self.slices = []
        names = {id(p): n for n, p in module.named_parameters()}
        for p, o in zip(params, offs):
            n = p.numel()
            view = self.data[o:o + n].view_as(p)
            view.copy_(p.data.to(dev))
            p.data = view
            p.grad = self.grad[o:o + n].view_as(p)
            p._mbk_grad_at = (self.grad, o, n)
            self.slices.append((names.get(id(p), "?"), o, n, tuple(p.shape)))
        self.params = params
        # "direct" parameters: their backward kernels write the gradient straight into the
        # flat slot (``grad_out``) and autograd adopts that view as .grad -- no zero fill of
        # the buffer, no AccumulateGrad add kernel per parameter
        # (only when the module says its backward will take that path on this device)
        ok = getattr(module, "direct_grad_ok", None)
        allow = bool(ok(dev)) if ok is not None else False
        self.direct = [allow and bool(getattr(p, "_mbk_direct_grad", False)) for p in params]

    def zero_grad(self):
        if not any(self.direct):
            zero_(self.grad)
        else:
            if not all(self.direct):
                zero_(self.grad)
            for p, d in zip(self.params, self.direct):
                if d:
                    p.grad = None
        # autograd may have replaced a .grad (e.g. after set_to_none elsewhere): re-bind views
        for p, d, (_, o, n, _) in zip(self.params, self.direct, self.slices):
            if not d and (p.grad is None or p.grad.data_ptr() != self.grad[o:].data_ptr()):
                p.grad = self.grad[o:o + n].view_as(p)

    def adopt_grads(self) -> int:
        """After backward: bind every direct parameter's .grad to its flat slot (copying a
        gradient autograd did not adopt in place, zeroing one that got none). Returns the
        number of such fix-ups (0 on the fast path)."""
        fixed = 0
        for p, d, (_, o, n, _) in zip(self.params, self.direct, self.slices):
            if not d:
                continue
            g = p.grad
            if g is not None and g.data_ptr() == self.grad[o:].data_ptr():
                continue
            slot = self.grad[o:o + n].view_as(p)
            if g is None:
                zero_(slot)
            else:
                slot.copy_(g)
            p.grad = slot
            fixed += 1
        return fixed

    def check_grad_views(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == self.grad[o:].data_ptr()
                   for p, (_, o, _, _) in zip(self.params, self.slices))


def grad_out(p: torch.Tensor) -> torch.Tensor:
    """fp32 buffer a backward kernel writes p's gradient into: p's flat gradient slot when p
    is a direct-gradient parameter awaiting its gradient (autograd then adopts the returned
    view as p.grad without a copy or an add), else a fresh tensor. A direct parameter must
    receive its gradient from exactly one autograd node per backward."""
    at = getattr(p, "_mbk_grad_at", None)
    if at is not None and p.grad is None and getattr(p, "_mbk_direct_grad", False):
        buf, o, n = at
        return buf[o:o + n].view(p.shape)
    return torch.empty(p.shape, dtype=torch.float32, device=p.device)


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
        self.m = zeros(flat.data.shape, device=flat.data.device)
        self.v = zeros(flat.data.shape, device=flat.data.device)
        self.step_count = 0
        self.shadow = torch.empty(flat.numel, dtype=torch.bfloat16, device=dev) if bf16_shadow else None
        self._partials = torch.empty(1024, dtype=torch.float32, device=dev)
        self._scale = full((2,), 1.0, device=dev)
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
