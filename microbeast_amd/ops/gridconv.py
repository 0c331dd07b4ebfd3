"""GridNet convolutions on the hand-written MFMA GEMM (``gemm.hip``), NHWC bf16.

GridNet (BASELINE config 2) has 3x3 convs of 27..256 channels and stride-2 transposed
convs. Both are expressed as GEMMs on our kernel, with im2col / col2im as pure data
movement:

* ``conv3x3``: NHWC im2col (K order ky, kx, ci) [B*H*W, 9*Cin] . W[Cout, 9*Cin]^T + b
  -> NHWC output, relu optionally fused into the GEMM epilogue;
* ``conv_transpose3x3s2`` (k3 s2 p1 op1): X[B*H*W, Cin] . Wt[Cout*9, Cin]^T -> per-pixel
  columns, scattered with ``fold`` into the 2H x 2W output (the transposed conv's
  definition), + bias (+ relu).

Gradients come from the GEMM's autograd (dA on the GEMM kernel, dW on the split-K kernel)
and the data-movement ops' own backward.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .gemm import gemm_nt


def conv3x3(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, relu: bool = False):
    """x NHWC bf16 [B, H, W, Cin] (Cin % 8 == 0 after padding the weight), w [Cout, Cin_w, 3, 3]
    (fp32 parameter; Cin_w <= Cin, zero-extended). Returns NHWC bf16 [B, H, W, Cout]."""
    B, H, W, C = x.shape
    if w.shape[1] < C:
        w = F.pad(w, (0, 0, 0, 0, 0, C - w.shape[1]))
    xp = F.pad(x, (0, 0, 1, 1, 1, 1))
    cols = torch.cat([xp[:, ky:ky + H, kx:kx + W, :] for ky in range(3) for kx in range(3)],
                     dim=-1)
    wk = w.permute(0, 2, 3, 1).reshape(w.shape[0], 9 * C)
    y = gemm_nt(cols.reshape(B * H * W, 9 * C), wk, b, relu=relu)
    return y.view(B, H, W, -1)


def maxpool3x3s2(x: torch.Tensor) -> torch.Tensor:
    """max_pool2d(3, 2, 1) of an NHWC tensor (channels-last kernel, no layout copy)."""
    y = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1)
    return y.permute(0, 2, 3, 1)


def conv_transpose3x3s2(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None,
                        relu: bool = False, nchw_out: bool = False):
    """ConvTranspose2d(k=3, stride=2, padding=1, output_padding=1) of NHWC bf16 x [B, H, W, Cin];
    w [Cin, Cout, 3, 3] (PyTorch ConvTranspose layout). Returns NHWC [B, 2H, 2W, Cout]
    (or NCHW with nchw_out)."""
    B, H, W, Cin = x.shape
    Cout = w.shape[1]
    wt = w.permute(1, 2, 3, 0).reshape(Cout * 9, Cin)  # rows (co, ky, kx)
    cols = gemm_nt(x.reshape(B * H * W, Cin), wt)  # [B*H*W, Cout*9]
    cols = cols.view(B, H * W, Cout * 9).transpose(1, 2)
    y = F.fold(cols.float(), output_size=(2 * H, 2 * W), kernel_size=3, stride=2, padding=1)
    if b is not None:
        y = y + b.view(1, -1, 1, 1)
    if relu:
        y = F.relu(y)
    y = y.to(torch.bfloat16)
    return y if nchw_out else y.permute(0, 2, 3, 1).contiguous()
