"""GridNet convolutions as shifted-row ("implicit im2col") MFMA GEMMs, NHWC bf16.

GridNet (BASELINE config 2, reference models/gridnet.py) stacks 3x3 convs of 27..256
channels, max-pools and stride-2 transposed convs (k3 s2 p1 op1). An explicit im2col
(9x the activation bytes) or col2im ``fold`` (fp32 columns of Cout*9 per pixel) costs far
more HBM traffic than the MFMA work itself, so neither is materialised here:

* ``conv3x3``: the input is zero-padded once to [B, H+2, W+2, C] and flattened to rows
  p = (b, y, x). At every padded position, out[p] = sum_t xp[p + s_t] . W_t with
  s_t = (ky-1)*(W+2) + (kx-1). That is ONE GEMM whose A operand reads, for the K block of
  tap t, rows shifted by s_t (``mbk_gemm_nt_taps``, gemm.hip). Bias and relu are fused in
  the epilogue, whose row remap writes only interior rows, straight to their NHWC
  position. Border outputs are computed but never stored (1.27x work at 16x16). In
  exchange, no A operand is ever materialised.
* ``conv_transpose3x3s2``: output pixel (2j+a, 2i+b) gets taps from input rows j / j+1
  only (sub-pixel decomposition). Each of the 4 phases (a, b) is a shifted-row GEMM of
  1, 2, 2 or 4 taps, whose epilogue remap writes the phase's stride-2 pixels of the NHWC
  output directly (no scatter copy).
* Backward: dX is one more shifted-row GEMM with negated shifts (all 9 taps, for the
  transposed conv across the 4 phase gradients). dW is the split-K kernel of fc.hip with
  shifted x rows (``mbk_fc_wgrad_taps``): all taps in one launch, with column chunks that
  span taps, so 32-channel layers fill whole 64-wide tiles. db is a column sum.

Channel counts are zero-padded to multiples of 32, so a 32-wide K step never straddles
two taps. Off-GPU, the same shifted-row maths runs in plain torch (``_taps_gemm_ref`` /
``_taps_wgrad_ref``), so the index maths is unit-tested on CPU against F.conv2d /
F.conv_transpose2d.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F

_BF = torch.bfloat16


def _ceil32(c: int) -> int:
    return -(-c // 32) * 32


def _pad_grid(x: torch.Tensor, cp: int) -> torch.Tensor:
    """NHWC [B, H, W, C] -> zero-padded [B*(H+2)*(W+2), cp] bf16 rows."""
    B, H, W, C = x.shape
    return F.pad(x.to(_BF), (0, cp - C, 1, 1, 1, 1)).reshape(B * (H + 2) * (W + 2), cp)


def _dx(B, H, W, cp, C, bases, shifts, bm):
    """input gradient [B, H, W, C] from a shifted-row GEMM over the padded gradient grid"""
    dx = torch.empty(B, H, W, cp, dtype=_BF, device=bm.device)
    taps_gemm(bases, shifts, bm, out=dx.view(-1, cp), remap=(H + 2, W + 2, H * W, W, 1, 1, 0, 0))
    return dx if C == cp else dx[..., :C].contiguous()


# ----------------------------------------------------------------------------- launchers
def _shift_rows(a: torch.Tensor, s: int) -> torch.Tensor:
    """rows r -> a[r + s], zero outside (reference semantics of a shifted A operand)."""
    out = torch.zeros_like(a)
    M = a.shape[0]
    lo, hi = max(0, -s), min(M, M - s)
    if hi > lo:
        out[lo:hi] = a[lo + s:hi + s]
    return out


def _remap_index(M, remap, device):
    """(src rows, dst rows) of the epilogue row remap (gemm.hip ATaps): interior rows of the
    padded grid -> b*ob + ((y-1)*sy + oy0)*ow + (x-1)*sx + ox0."""
    Hp, Wp, ob, ow, sy, sx, oy0, ox0 = remap
    m = torch.arange(M, device=device)
    x, t = m % Wp, m // Wp
    y, b = t % Hp, t // Hp
    keep = (y > 0) & (y < Hp - 1) & (x > 0) & (x < Wp - 1)
    m, x, y, b = m[keep], x[keep], y[keep], b[keep]
    return m, b * ob + ((y - 1) * sy + oy0) * ow + (x - 1) * sx + ox0


def _taps_gemm_ref(bases, shifts, b, bias, relu, out_dtype, out=None, remap=None):
    tk = bases[0].shape[1]
    acc = None
    for t, (a, s) in enumerate(zip(bases, shifts)):
        part = _shift_rows(a.float(), s) @ b[:, t * tk:(t + 1) * tk].float().t()
        acc = part if acc is None else acc + part
    if bias is not None:
        acc = acc + bias.float()
    if relu:
        acc = acc.clamp_min(0)
    if remap is None:
        if out is None:
            return acc.to(out_dtype)
        out.copy_(acc)
        return out
    src, dst = _remap_index(acc.shape[0], remap, acc.device)
    out[dst] = acc[src].to(out.dtype)
    return out


def taps_gemm(bases, shifts, b, bias=None, relu=False, out_dtype=_BF, out=None, remap=None):
    """C[M, N] = sum_t A_t[m + shift_t] . B[:, t*tk:(t+1)*tk]^T (+bias)(+relu).
    bases: list of [M, tk] bf16 (contiguous, tk % 32 == 0); b: [N, ntap*tk] bf16.
    remap (Hp, Wp, ob, ow, sy, sx, oy0, ox0): write only the interior rows of the padded
    grid, each to its output row (see gemm.hip ATaps); ``out`` is then required
    ([rows, N] with unit column stride)."""
    M, tk = bases[0].shape
    assert tk % 32 == 0 and b.shape[1] == len(bases) * tk and len(bases) <= 9
    assert remap is None or out is not None
    if not b.is_cuda:
        return _taps_gemm_ref(bases, shifts, b, bias, relu, out_dtype, out, remap)
    from .. import _native as N
    for a in bases:
        assert a.shape == (M, tk) and a.is_contiguous() and a.dtype == _BF
    b = b.to(_BF).contiguous()
    if out is None:
        out = torch.empty(M, b.shape[0], dtype=out_dtype, device=b.device)
    assert out.stride(-1) == 1 and out.shape[-1] == b.shape[0]
    if remap is not None:
        Hp, Wp, ob, ow, sy, sx, oy0, ox0 = remap
        last = (M // (Hp * Wp) - 1) * ob + ((Hp - 3) * sy + oy0) * ow + (Wp - 3) * sx + ox0
        assert M % (Hp * Wp) == 0 and last < out.shape[0], "remap writes out of bounds"
    ptrs = (ctypes.c_void_p * 9)(*[a.data_ptr() for a in bases])
    sh = (ctypes.c_int * 9)(*shifts)
    rm = (ctypes.c_int * 8)(*remap) if remap is not None else None
    if bias is not None:
        bias = bias.float().contiguous()
    N.check(N.kernels().mbk_gemm_nt_taps(ptrs, sh, len(bases), tk, b.data_ptr(),
                                         out.data_ptr(), N.ptr(bias), M, b.shape[0], tk,
                                         b.shape[1], out.stride(-2), int(relu),
                                         int(out.dtype == _BF), 0, rm, N.stream_ptr()),
            "gemm_nt_taps")
    return out


def _taps_wgrad_ref(g, x, shifts):
    return torch.cat([g.float().t() @ _shift_rows(x.float(), s) for s in shifts], dim=1)


def taps_wgrad(g: torch.Tensor, x: torch.Tensor, shifts) -> torch.Tensor:
    """fp32 [O, ntap*I]: block t = g[N, O]^T . x[n + shift_t] (x rows outside [0, N) zero)."""
    n, o = g.shape
    i = x.shape[1]
    if not g.is_cuda:
        return _taps_wgrad_ref(g, x, shifts)
    from .. import _native as N
    k = N.kernels()
    g = g.to(_BF).contiguous()
    x = x.to(_BF).contiguous()
    nt = len(shifts)
    nparts = k.mbk_fc_wgrad_parts(n, o, i * nt)
    scratch = torch.empty((nparts + (nparts + 31) // 32) * o * i * nt, dtype=torch.float32,
                          device=g.device)
    out = torch.empty(o, nt * i, dtype=torch.float32, device=g.device)
    sh = (ctypes.c_int * 9)(*shifts)
    N.check(k.mbk_fc_wgrad_taps(g.data_ptr(), x.data_ptr(), n, o, i, sh, nt, scratch.data_ptr(),
                                nparts, out.data_ptr(), 0, N.stream_ptr()), "fc_wgrad_taps")
    return out


# ----------------------------------------------------------------------------- conv 3x3
def _conv_shifts(W: int):
    Wp = W + 2
    return [(ky - 1) * Wp + (kx - 1) for ky in range(3) for kx in range(3)]


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        B, H, W, C = x.shape
        Cout, Cw = w.shape[:2]
        cp = _ceil32(max(C, Cw))
        xp = _pad_grid(x, cp)
        wk = F.pad(w.detach(), (0, 0, 0, 0, 0, cp - Cw)).permute(0, 2, 3, 1)
        wk = wk.reshape(Cout, 9 * cp).to(_BF).contiguous()  # tap-major K (ky, kx, ci)
        sh = _conv_shifts(W)
        y = torch.empty(B, H, W, Cout, dtype=_BF, device=x.device)
        taps_gemm([xp] * 9, sh, wk, b.detach() if b is not None else None, relu,
                  out=y.view(-1, Cout), remap=(H + 2, W + 2, H * W, W, 1, 1, 0, 0))
        ctx.save_for_backward(xp, wk, y if relu else None)
        ctx.meta = (B, H, W, C, Cw, cp, relu, b is not None, w.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        xp, wk, y = ctx.saved_tensors
        B, H, W, C, Cw, cp, relu, has_b, wdt = ctx.meta
        Cout = wk.shape[0]
        g = gy.to(_BF)
        if relu:
            g = g * (y > 0)
        cop = _ceil32(Cout)
        gp = _pad_grid(g, cop)  # zero border: border outputs get no gradient
        sh = _conv_shifts(W)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            # dxp[q] = sum_t g[q - s_t] . W_t : B operand [cp, 9*cop], block t = W_t^T
            wt = wk.view(Cout, 9, cp).permute(2, 1, 0)  # [cp, 9, Cout]
            wt = F.pad(wt, (0, cop - Cout)).reshape(cp, 9 * cop).contiguous()
            gx = _dx(B, H, W, cp, C, [gp] * 9, [-s for s in sh], wt)
        if ctx.needs_input_grad[1]:
            dw = taps_wgrad(gp, xp, sh)[:Cout]  # [Cout, 9*cp]
            gw = dw.view(Cout, 3, 3, cp).permute(0, 3, 1, 2)[:, :Cw].contiguous().to(wdt)
        if has_b and ctx.needs_input_grad[2]:
            gb = g.float().sum((0, 1, 2))
        return gx, gw, gb, None


def conv3x3(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, relu: bool = False):
    """Conv2d(k=3, padding=1) of NHWC x [B, H, W, Cin] (bf16), w [Cout, Cin_w, 3, 3] (fp32
    parameter; Cin_w <= Cin, zero-extended). Returns NHWC bf16 [B, H, W, Cout]."""
    return _Conv3x3.apply(x, w, b, relu)


def maxpool3x3s2(x: torch.Tensor) -> torch.Tensor:
    """max_pool2d(3, 2, 1) of an NHWC tensor (channels-last kernel, no layout copy)."""
    y = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1)
    return y.permute(0, 2, 3, 1)


# ----------------------------------------------------------------------------- transposed conv
# output row 2j + a receives kernel row ky from input row j + dy:
#   a = 0: (ky=1, dy=0);  a = 1: (ky=0, dy=1), (ky=2, dy=0)   (k3 s2 p1 op1)
_PH = {0: ((1, 0),), 1: ((0, 1), (2, 0))}


def _phase_taps(W: int):
    """[(a, b, [(ky, kx, shift), ...])] over the 4 output phases; 9 taps in total."""
    Wp = W + 2
    out = []
    for a in (0, 1):
        for b in (0, 1):
            out.append((a, b, [(ky, kx, dy * Wp + dx) for ky, dy in _PH[a] for kx, dx in _PH[b]]))
    return out


class _ConvT3x3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        B, H, W, Cin = x.shape
        Cout = w.shape[1]
        cip = _ceil32(Cin)
        xp = _pad_grid(x, cip)
        wb = F.pad(w.detach(), (0, 0, 0, 0, 0, 0, 0, cip - Cin)).to(_BF)  # [cip, Cout, 3, 3]
        y = torch.empty(B, 2 * H, 2 * W, Cout, dtype=_BF, device=x.device)
        bias = b.detach() if b is not None else None
        for a, bb, taps in _phase_taps(W):
            bm = torch.cat([wb[:, :, ky, kx].t() for ky, kx, _ in taps], dim=1).contiguous()
            taps_gemm([xp] * len(taps), [s for _, _, s in taps], bm, bias, relu,
                      out=y.view(-1, Cout), remap=(H + 2, W + 2, 4 * H * W, 2 * W, 2, 2, a, bb))
        ctx.save_for_backward(xp, wb, y if relu else None)
        ctx.meta = (B, H, W, Cin, cip, relu, b is not None, w.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        xp, wb, y = ctx.saved_tensors
        B, H, W, Cin, cip, relu, has_b, wdt = ctx.meta
        Cout = wb.shape[1]
        g = gy.to(_BF)
        if relu:
            g = g * (y > 0)
        cop = _ceil32(Cout)
        phases = _phase_taps(W)
        gps = [_pad_grid(g[:, a::2, bb::2, :], cop) for a, bb, _ in phases]
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            # dxp[q] = sum_{phase, tap} g_phase[q - s] . W[:, :, ky, kx]^T, one 9-tap GEMM
            bases, shifts, blocks = [], [], []
            for gp, (_, _, taps) in zip(gps, phases):
                for ky, kx, s in taps:
                    bases.append(gp)
                    shifts.append(-s)
                    blocks.append(F.pad(wb[:, :, ky, kx], (0, cop - Cout)))  # [cip, cop]
            gx = _dx(B, H, W, cip, Cin, bases, shifts, torch.cat(blocks, dim=1).contiguous())
        if ctx.needs_input_grad[1]:
            gw = torch.zeros(cip, Cout, 3, 3, dtype=torch.float32, device=g.device)
            for gp, (_, _, taps) in zip(gps, phases):
                dw = taps_wgrad(gp, xp, [s for _, _, s in taps])[:Cout]  # [Cout, ntap*cip]
                for t, (ky, kx, _) in enumerate(taps):
                    gw[:, :, ky, kx] = dw[:, t * cip:(t + 1) * cip].t()
            gw = gw[:Cin].contiguous().to(wdt)
        if has_b and ctx.needs_input_grad[2]:
            gb = g.float().sum((0, 1, 2))
        return gx, gw, gb, None


def conv_transpose3x3s2(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None,
                        relu: bool = False, nchw_out: bool = False):
    """ConvTranspose2d(k=3, stride=2, padding=1, output_padding=1) of NHWC bf16 x [B, H, W, Cin];
    w [Cin, Cout, 3, 3] (PyTorch ConvTranspose layout). Returns NHWC [B, 2H, 2W, Cout]
    (or an NCHW view with nchw_out)."""
    y = _ConvT3x3s2.apply(x, w, b, relu)
    return y.permute(0, 3, 1, 2) if nchw_out else y
