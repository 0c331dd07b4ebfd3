"""Hand-written MFMA GEMM (``gemm.hip``) with autograd.

``gemm_nt(a, b, bias, relu)`` = relu?(a @ b.T + bias) for bf16 ``a`` [M, K] and ``b``
[N, K], fp32 accumulation, bf16 result. Backward:

* dA = dC . B: the same kernel against B^T (B is a weight, a few hundred KB),
* dB = dC^T . A: the split-K kernel of ``fc.hip`` (``ops.linear.weight_grad``), fp32,
* dbias = column sums of dC.

Used by the trunk-tail Linear layers in training (no vendor GEMM on the hot path,
SURVEY §7.4 hard part 6) and by the GridNet convolutions (im2col . W^T).
"""
from __future__ import annotations

import torch

from .. import _native as N


def gemm_nt_raw(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None,
                relu: bool = False, out: torch.Tensor | None = None,
                out_dtype=torch.bfloat16, accumulate: bool = False) -> torch.Tensor:
    """No-grad launch. a [M,K] / b [N,K] bf16 with K-contiguous rows (K % 8 == 0)."""
    assert a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
    assert a.shape[1] == b.shape[1]
    K = a.shape[1]
    if K % 8 or a.stride(1) != 1 or b.stride(1) != 1 or a.stride(0) % 8 or b.stride(0) % 8:
        # the kernel reads 8-element K vectors: zero-pad K (adds nothing to the products)
        kp = -(-K // 8) * 8
        a = torch.nn.functional.pad(a, (0, kp - K))
        b = torch.nn.functional.pad(b, (0, kp - K))
    M, K = a.shape
    Nn = b.shape[0]
    if out is None:
        out = torch.empty(M, Nn, dtype=out_dtype, device=a.device)
    assert out.stride(1) == 1
    if bias is not None:
        bias = bias.float().contiguous()
    N.check(N.kernels().mbk_gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), N.ptr(bias), M,
                                    Nn, K, a.stride(0), b.stride(0), out.stride(0), int(relu),
                                    int(out.dtype == torch.bfloat16), int(accumulate),
                                    N.stream_ptr()), "gemm_nt")
    return out


class _GemmNT(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, bias, relu):
        # the bf16 cast of b happens here (not as an autograd node), so its gradient
        # comes back at b's own precision (fp32 master weights)
        bc = b.to(torch.bfloat16)
        if bc.stride(-1) != 1:
            bc = bc.contiguous()
        y = gemm_nt_raw(a, bc, bias, relu)
        ctx.relu = relu
        ctx.has_bias = bias is not None
        ctx.save_for_backward(a, bc, y if relu else None)
        ctx.b_dtype = b.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        from .linear import weight_grad
        a, b, y = ctx.saved_tensors
        g = g.to(torch.bfloat16)
        if ctx.relu:
            g = g * (y > 0)
        g = g.contiguous()
        ga = gb = gbias = None
        if ctx.needs_input_grad[0]:
            ga = gemm_nt_raw(g, b.t().contiguous())
        if ctx.needs_input_grad[1]:
            gb = weight_grad(g, a).to(ctx.b_dtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gbias = g.float().sum(0)
        return ga, gb, gbias, None


def gemm_nt(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None,
            relu: bool = False) -> torch.Tensor:
    """relu?(a @ b.T + bias): bf16 in / out, fp32 accumulate, differentiable."""
    a = a.to(torch.bfloat16)
    if a.stride(-1) != 1:
        a = a.contiguous()
    return _GemmNT.apply(a, b, bias, relu)
