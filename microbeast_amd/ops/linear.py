"""Dense layers of the trunk tail (``network.5`` and ``critic``) with a split-K weight grad.

Reference: nn.Linear(32*h/8*w/8, 256) + ReLU and the critic nn.Linear(256, 1)
(model.py:119-137). On the learner batch (T+1)*B ~ 266K rows these GEMMs are tiny in
FLOPs but the weight gradient dW = g^T x reduces over K = 266K with only a handful
of output tiles; the BLAS heuristics pick a 4-workgroup kernel for it (0.57 ms per
update measured, profiles/06_*), and batched split-K through aten::bmm(out_dtype=fp32)
blocks the host for milliseconds. Here dW comes from the split-K MFMA kernel in
``csrc/kernels/fc.hip`` (fp32 partials, deterministic reduce, no host sync).

The input may be the conv trunk's NHWC output flattened as-is: ``nhwc=(C, H, W)``
permutes the weight's input columns from the reference's NCHW flatten order
instead of copying the activations.
"""
from __future__ import annotations

import torch

_MIN_ROWS = 4096


def weight_grad(g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """fp32 [O, I] = g[N, O]^T @ x[N, I] (bf16 inputs), split over K = N (fc.hip)."""
    n, o = g.shape
    i = x.shape[1]
    if not g.is_cuda or n < _MIN_ROWS or i % 8:
        return g.t().float() @ x.float()
    from .. import _native as N
    k = N.kernels()
    g = g.contiguous().to(torch.bfloat16)
    x = x.contiguous().to(torch.bfloat16)
    nparts = k.mbk_fc_wgrad_parts(n, o, i)
    scratch = torch.empty((nparts + (nparts + 31) // 32) * o * i, dtype=torch.float32,
                          device=g.device)
    out = torch.empty(o, i, dtype=torch.float32, device=g.device)
    N.check(k.mbk_fc_wgrad(g.data_ptr(), x.data_ptr(), n, o, i, scratch.data_ptr(), nparts,
                           out.data_ptr(), 0, N.stream_ptr()), "fc_wgrad")
    return out


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        wc = w.to(x.dtype)
        ctx.save_for_backward(x, wc)
        ctx.w_dtype = w.dtype
        if x.is_cuda and x.dtype == torch.bfloat16:
            from .gemm import gemm_nt_raw  # hand-written MFMA GEMM (gemm.hip; pads K % 8)
            return gemm_nt_raw(x.reshape(-1, x.shape[-1]), wc.contiguous(),
                               b).view(*x.shape[:-1], wc.shape[0])
        return torch.nn.functional.linear(x, wc, b.to(x.dtype) if b is not None else None)

    @staticmethod
    def backward(ctx, g):
        x, wc = ctx.saved_tensors
        g = g.contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            if g.is_cuda and g.dtype == torch.bfloat16:
                from .gemm import gemm_nt_raw  # K = out_features (1 for the critic): padded
                gx = gemm_nt_raw(g.reshape(-1, g.shape[-1]), wc.t().contiguous())
                gx = gx.view(*g.shape[:-1], wc.shape[1])
            else:
                gx = g @ wc
        gw = weight_grad(g, x).to(ctx.w_dtype) if ctx.needs_input_grad[1] else None
        gb = g.float().sum(0) if ctx.needs_input_grad[2] else None
        return gx, gw, gb


def nhwc_weight(w: torch.Tensor, nhwc: tuple[int, int, int] | None) -> torch.Tensor:
    """Permute a Linear weight's input columns from NCHW to NHWC flatten order."""
    if nhwc is None:
        return w
    c, h, wd = nhwc
    return w.view(w.shape[0], c, h, wd).permute(0, 2, 3, 1).reshape(w.shape[0], -1)


def linear(x: torch.Tensor, layer: torch.nn.Linear, dtype=torch.bfloat16,
           nhwc: tuple[int, int, int] | None = None, cached=None) -> torch.Tensor:
    """``layer(x)`` computed in ``dtype`` with the split-K weight gradient.
    cached: (weight, bias) already converted (inference with prepacked weights)."""
    if cached is not None:
        if x.is_cuda and dtype == torch.bfloat16:
            from .gemm import gemm_nt_raw
            return gemm_nt_raw(x.to(dtype).reshape(-1, x.shape[-1]), cached[0], cached[1])
        return torch.nn.functional.linear(x.to(dtype), cached[0], cached[1])
    return _Linear.apply(x.to(dtype), nhwc_weight(layer.weight, nhwc), layer.bias)
