"""GridNet layers on shifted-row ("implicit im2col") MFMA GEMMs over zero-padded NHWC grids.

GridNet (BASELINE config 2, ``models/gridnet.py``) stacks conv3x3 + relu + max-pool(3, 2, 1)
encoder layers of 27..256 channels, stride-2 transposed convs (k3 s2 p1 op1) and a two-layer
critic. An explicit im2col (9x the activation bytes) or col2im ``fold`` (fp32 columns of
Cout*9 per pixel) costs far more HBM traffic than the MFMA work itself, so neither exists:

* Activations live on zero-padded grids ``[B, H+2, W+2, C]`` (bf16, border = 0), flattened
  to rows p = (b, y, x). At every padded position, conv3x3 out[p] = sum_t xp[p + s_t] . W_t
  with s_t = (ky-1)*(W+2) + (kx-1): ONE GEMM whose A operand reads, for the K block of tap t,
  rows shifted by s_t (``mbk_gemm_nt_taps``, gemm.hip). Bias and relu are fused in the
  epilogue, whose row remap writes straight to the output's NHWC position; with
  ``zero_border`` it also writes the zero border of a padded output grid, so no layer ever
  pads, crops or scatters a tensor.
* conv3x3 + relu + max-pool: the pool (``mbk_pool_fwd``, gridnet.hip) reads the conv output
  and writes the next layer's padded grid plus a uint8 argmax; its backward
  (``mbk_pool_bwd_grid``) routes the pooled gradient (relu mask = pooled > 0) to the argmax
  and writes the conv's padded output-gradient grid, the operand of its dgrad / wgrad GEMMs.
* Transposed conv: output pixel (2j+a, 2i+b) gets taps from input rows j / j+1 only
  (sub-pixel decomposition). Each of the 4 phases (a, b) is a shifted-row GEMM of 1, 2, 2 or
  4 taps whose epilogue writes the phase's stride-2 pixels of the padded output grid (or of
  the cropped cell-major logits for the last layer). Its backward gathers the output
  gradient (relu-masked, or straight from the masked-cell head's dlogits) into 4 padded
  phase grids (``mbk_grid_gather``): dX is one 9-tap GEMM over them, dW four shifted
  split-K GEMMs (fc.hip ``mbk_fc_wgrad_taps``).
* The observation bit planes are expanded into the first padded grid by ``mbk_bits_grid``.
* Weights: every GEMM operand layout (tap-major, channel-padded, transposed for dgrad, the
  critic's NCHW->NHWC column order) is gathered from the fp32 parameters by ONE
  ``mbk_map_gather`` launch per forward through index maps built once per model; weight
  gradients come back into the parameters' own layouts the same way. Bias gradients are
  deterministic column sums (``mbk_colsum``), the critic's output layer has its own
  backward (``mbk_value_bwd``).

Channel counts are zero-padded to multiples of 32, so a 32-wide K step never straddles two
taps. Off-GPU every launcher runs a plain-torch emulation of the same index maths, so the
whole layer stack is unit-tested on CPU against F.conv2d / F.max_pool2d /
F.conv_transpose2d (tests/test_gridconv.py); tests/test_gpu_gridconv.py runs the kernels.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

_BF = torch.bfloat16
_BIG = 1 << 30


def _ceil32(c: int) -> int:
    return -(-c // 32) * 32


def _N():
    from .. import _native as N
    return N


# ============================================================================ launchers
# Every launcher takes device tensors; off-GPU it emulates the kernel in torch.

def _shift_rows(a: torch.Tensor, s: int) -> torch.Tensor:
    """rows r -> a[r + s], zero outside (reference semantics of a shifted A operand)."""
    out = torch.zeros_like(a)
    M = a.shape[0]
    lo, hi = max(0, -s), min(M, M - s)
    if hi > lo:
        out[lo:hi] = a[lo + s:hi + s]
    return out


def remap(Hp, Wp, ob, ow, sy=1, sx=1, oy0=0, ox0=0, lim=(_BIG, _BIG), zero_border=False):
    """Epilogue row remap of ``taps_gemm`` (gemm.hip ATaps): GEMM row m = (b, y, x) of the
    padded input grid [*, Hp, Wp] -> output row b*ob + Y*ow + X with
    (Y, X) = ((y-1)*sy + oy0, (x-1)*sx + ox0); outputs outside [0, lim) are dropped; border
    rows are dropped, or write zeros with ``zero_border``."""
    return (Hp, Wp, ob, ow, sy, sx, oy0, ox0, lim[0], lim[1], int(zero_border))


def _remap_index(M, rm, device):
    """(src rows, dst rows, zero flags) of a remap (emulation)."""
    Hp, Wp, ob, ow, sy, sx, oy0, ox0, lh, lw, zb = rm
    m = torch.arange(M, device=device)
    x, t = m % Wp, m // Wp
    y, b = t % Hp, t // Hp
    border = (y == 0) | (y == Hp - 1) | (x == 0) | (x == Wp - 1)
    Y, X = (y - 1) * sy + oy0, (x - 1) * sx + ox0
    keep = (~border | bool(zb)) & (Y >= 0) & (Y < lh) & (X >= 0) & (X < lw)
    return m[keep], (b * ob + Y * ow + X)[keep], border[keep]


def _remap_last_row(M, rm) -> int:
    Hp, Wp, ob, ow, sy, sx, oy0, ox0, lh, lw, zb = rm
    ylast, xlast = (Hp - 1, Wp - 1) if zb else (Hp - 2, Wp - 2)
    Y = min(lh - 1, (ylast - 1) * sy + oy0)
    X = min(lw - 1, (xlast - 1) * sx + ox0)
    return (M // (Hp * Wp) - 1) * ob + Y * ow + X


def _taps_gemm_ref(bases, shifts, b, bias, relu, out_dtype, out=None, rm=None):
    tk = bases[0].shape[1]
    acc = None
    for t, (a, s) in enumerate(zip(bases, shifts)):
        part = _shift_rows(a.float(), s) @ b[:, t * tk:(t + 1) * tk].float().t()
        acc = part if acc is None else acc + part
    if bias is not None:
        acc = acc + bias.float()
    if relu:
        acc = acc.clamp_min(0)
    if rm is None:
        if out is None:
            return acc.to(out_dtype)
        out.copy_(acc)
        return out
    src, dst, zero = _remap_index(acc.shape[0], rm, acc.device)
    vals = acc[src]
    vals[zero] = 0
    out[dst] = vals.to(out.dtype)
    return out


def taps_gemm(bases, shifts, b, bias=None, relu=False, out_dtype=None, out=None, rm=None):
    """C[M, N] = sum_t A_t[m + shift_t] . B[:, t*tk:(t+1)*tk]^T (+bias)(+relu).
    bases: list of [M, tk] bf16 (contiguous, tk % 32 == 0); b: [N, ntap*tk] bf16.
    rm: ``remap(...)`` tuple; ``out`` is then required ([rows, N], unit column stride)."""
    M, tk = bases[0].shape
    assert tk % 32 == 0 and b.shape[1] == len(bases) * tk and len(bases) <= 9
    assert rm is None or out is not None
    if rm is not None:
        assert M % (rm[0] * rm[1]) == 0 and _remap_last_row(M, rm) < out.shape[0], \
            "remap writes out of bounds"
    out_dtype = out_dtype or _BF
    if not b.is_cuda:
        return _taps_gemm_ref(bases, shifts, b, bias, relu, out_dtype, out, rm)
    N = _N()
    for a in bases:
        assert a.shape == (M, tk) and a.is_contiguous() and a.dtype == _BF
    assert b.dtype == _BF and b.is_contiguous()
    if out is None:
        out = torch.empty(M, b.shape[0], dtype=out_dtype, device=b.device)
    assert out.stride(-1) == 1 and out.shape[-1] == b.shape[0]
    ptrs = (ctypes.c_void_p * 9)(*[a.data_ptr() for a in bases])
    sh = (ctypes.c_int * 9)(*shifts)
    rma = (ctypes.c_int * 11)(*rm) if rm is not None else None
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    N.check(N.kernels().mbk_gemm_nt_taps(ptrs, sh, len(bases), tk, b.data_ptr(),
                                         out.data_ptr(), N.ptr(bias), M, b.shape[0], tk,
                                         b.shape[1], out.stride(-2), int(relu),
                                         int(out.dtype == _BF), 0, rma, N.stream_ptr()),
            "gemm_nt_taps")
    return out


def _taps_wgrad_ref(g, x, shifts):
    return torch.cat([g.float().t() @ _shift_rows(x.float(), s) for s in shifts], dim=1)


def taps_wgrad(g: torch.Tensor, x: torch.Tensor, shifts, out: torch.Tensor | None = None):
    """fp32 [O, ntap*I]: block t = g[N, O]^T . x[n + shift_t] (x rows outside [0, N) zero)."""
    n, o = g.shape
    i = x.shape[1]
    nt = len(shifts)
    if out is None:
        out = torch.empty(o, nt * i, dtype=torch.float32, device=g.device)
    if not g.is_cuda:
        out.view(-1).copy_(_taps_wgrad_ref(g, x, shifts).reshape(-1))
        return out
    N = _N()
    k = N.kernels()
    assert g.dtype == _BF and x.dtype == _BF and g.is_contiguous() and x.is_contiguous()
    assert out.is_contiguous() and out.numel() == o * nt * i
    nparts = k.mbk_fc_wgrad_parts(n, o, i * nt)
    scratch = torch.empty((nparts + (nparts + 31) // 32) * o * i * nt, dtype=torch.float32,
                          device=g.device)
    sh = (ctypes.c_int * 9)(*shifts)
    N.check(k.mbk_fc_wgrad_taps(g.data_ptr(), x.data_ptr(), n, o, i, sh, nt, scratch.data_ptr(),
                                nparts, out.data_ptr(), 0, N.stream_ptr()), "fc_wgrad_taps")
    return out


def gemm_nt(a, b, bias=None, relu=False, out_dtype=None):
    """relu?(a . b^T + bias) on gemm.hip (no autograd): a [M, K], b [N, K] bf16, K % 8 == 0."""
    out_dtype = out_dtype or _BF
    assert a.shape[1] == b.shape[1] and a.shape[1] % 8 == 0
    if not a.is_cuda:
        y = a.float() @ b.float().t()
        if bias is not None:
            y = y + bias
        return (y.clamp_min(0) if relu else y).to(out_dtype)
    N = _N()
    assert a.is_contiguous() and b.is_contiguous() and a.dtype == _BF and b.dtype == _BF
    out = torch.empty(a.shape[0], b.shape[0], dtype=out_dtype, device=a.device)
    N.check(N.kernels().mbk_gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), N.ptr(bias),
                                    a.shape[0], b.shape[0], a.shape[1], a.shape[1], b.shape[1],
                                    b.shape[0], int(relu), int(out_dtype == _BF), 0,
                                    N.stream_ptr()), "gemm_nt")
    return out


def bits_grid(bits: torch.Tensor, h: int, w: int, Hp: int, Wp: int) -> torch.Tensor:
    """int32 bit-plane obs [n, h*w] -> padded bf16 grid [n, Hp, Wp, 32] (planes = bits)."""
    n = bits.shape[0]
    if not bits.is_cuda:
        sh = torch.arange(32, device=bits.device, dtype=torch.int32)
        x = ((bits.reshape(n, h, w, 1) >> sh) & 1).to(_BF)
        return F.pad(x, (0, 0, 1, Wp - w - 1, 1, Hp - h - 1))
    N = _N()
    assert bits.dtype == torch.int32 and bits.is_contiguous()
    out = torch.empty(n, Hp, Wp, 32, dtype=_BF, device=bits.device)
    N.check(N.kernels().mbk_bits_grid(bits.data_ptr(), n, h, w, Hp, Wp, out.data_ptr(),
                                      N.stream_ptr()), "bits_grid")
    return out


def pool_fwd(y: torch.Tensor, plain: bool, padded: bool):
    """max_pool(3, 2, 1) of NHWC y [B, H, W, C] -> (plain [B, Ho, Wo, C] | None,
    padded [B, Ho+2, Wo+2, C] | None, argmax uint8 [B, Ho, Wo, C] = ky*3+kx)."""
    B, H, W, C = y.shape
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    if not y.is_cuda:
        yp = F.pad(y.float(), (0, 0, 1, 1, 1, 1), value=float("-inf"))
        taps = torch.stack([yp[:, ky:ky + 2 * Ho:2, kx:kx + 2 * Wo:2]
                            for ky in range(3) for kx in range(3)], 0)
        mx, idx = taps.max(0)  # first maximum on ties (ATen's scan order)
        mx = mx.to(_BF)
        pp = F.pad(mx, (0, 0, 1, 1, 1, 1)) if padded else None
        return (mx if plain else None), pp, idx.to(torch.uint8)
    N = _N()
    assert y.is_contiguous() and y.dtype == _BF and C % 8 == 0
    out = torch.empty(B, Ho, Wo, C, dtype=_BF, device=y.device) if plain else None
    pp = torch.empty(B, Ho + 2, Wo + 2, C, dtype=_BF, device=y.device) if padded else None
    idx = torch.empty(B, Ho, Wo, C, dtype=torch.uint8, device=y.device)
    N.check(N.kernels().mbk_pool_fwd(y.data_ptr(), B, H, W, C, N.ptr(out), N.ptr(pp),
                                     idx.data_ptr(), N.stream_ptr()), "pool_fwd")
    return out, pp, idx


def pool_bwd(g1, pad1, g2, pad2, pooled, padp, idx, H: int, W: int) -> torch.Tensor:
    """Gradient of relu + max-pool -> padded conv-output gradient [B, H+2, W+2, C] (bf16).
    g1 / g2 (g2 optional): pooled-output gradients on plain (pad=0) or padded (pad=1) grids;
    pooled: the pool output (relu mask pooled > 0) on a plain or padded grid."""
    B, Ho, Wo, C = idx.shape
    if not idx.is_cuda:
        def plain(t, p):
            return t[:, 1:-1, 1:-1] if p else t
        g = plain(g1, pad1).float()
        if g2 is not None:
            g = g + plain(g2, pad2).float()
        g = g * (plain(pooled, padp).float() > 0)
        dy = torch.zeros(B, H + 2, W + 2, C, dtype=torch.float32)
        for t in range(9):
            ky, kx = divmod(t, 3)
            dy[:, ky:ky + 2 * Ho:2, kx:kx + 2 * Wo:2] += g * (idx == t)
        dy[:, 0] = 0
        dy[:, -1] = 0
        dy[:, :, 0] = 0
        dy[:, :, -1] = 0
        return dy.to(_BF)
    N = _N()
    for t in (g1, g2, pooled):
        assert t is None or (t.is_contiguous() and t.dtype == _BF)
    dy = torch.empty(B, H + 2, W + 2, C, dtype=_BF, device=idx.device)
    N.check(N.kernels().mbk_pool_bwd_grid(g1.data_ptr(), int(pad1), N.ptr(g2), int(pad2),
                                          pooled.data_ptr(), int(padp), idx.data_ptr(), B, H, W,
                                          C, dy.data_ptr(), N.stream_ptr()), "pool_bwd_grid")
    return dy


def grid_gather(src, sgeo, mask, mgeo, S: int, B: int, Hd: int, Wd: int, Cd: int):
    """dst [S*S, B, Hd+2, Wd+2, Cd] bf16, zero border / channel pad:
    dst[a*S+c, b, y, x, ch] = src(b, S*(y-1)+a, S*(x-1)+c, ch) * (mask(..) > 0).
    sgeo = (offset, sb, sy, sx, Hv, Wv, Cs) element strides of src (channels unit stride;
    only (Y, X) < (Hv, Wv), ch < Cs are read); mgeo = (offset, mb, my, mx) of mask."""
    off, sb, sy, sx, Hv, Wv, Cs = sgeo
    if not src.is_cuda:
        dst = torch.zeros(S * S, B, Hd + 2, Wd + 2, Cd, dtype=torch.float32)
        flat = src.reshape(-1).float()
        mflat = mask.reshape(-1).float() if mask is not None else None
        b = torch.arange(B)[:, None, None, None]
        ch = torch.arange(Cs)[None, None, None, :]
        for ph in range(S * S):
            a, c = divmod(ph, S)
            Y = (S * torch.arange(Hd) + a)[None, :, None, None]
            X = (S * torch.arange(Wd) + c)[None, None, :, None]
            ok = (Y < Hv) & (X < Wv)
            v = flat[(off + b * sb + Y.clamp(max=Hv - 1) * sy + X.clamp(max=Wv - 1) * sx + ch)]
            if mask is not None:
                mo, mb, my, mx = mgeo
                mv = mflat[mo + b * mb + Y.clamp(max=Hv - 1) * my + X.clamp(max=Wv - 1) * mx + ch]
                v = v * (mv > 0)
            dst[ph, :, 1:Hd + 1, 1:Wd + 1, :Cs] = v * ok
        return dst.to(_BF)
    N = _N()
    assert src.is_contiguous() and (mask is None or mask.is_contiguous())
    esz = src.element_size()
    dst = torch.empty(S * S, B, Hd + 2, Wd + 2, Cd, dtype=_BF, device=src.device)
    mo, mb, my, mx = mgeo if mask is not None else (0, 0, 0, 0)
    geo = (ctypes.c_int * 14)(int(src.dtype == torch.float32), sb, sy, sx, Hv, Wv, Cs, mb, my,
                              mx, S, B, Hd, Wd)
    mptr = mask.data_ptr() + 2 * mo if mask is not None else None
    N.check(N.kernels().mbk_grid_gather(src.data_ptr() + esz * off, mptr, geo, dst.data_ptr(), Cd,
                                        N.stream_ptr()), "grid_gather")
    return dst


def colsum(x: torch.Tensor, C: int, out0: torch.Tensor, c0: int | None = None,
           out1: torch.Tensor | None = None):
    """Column sums of the first C columns of 2-D x (bf16 / fp32) into out0[:c0] and
    out1[:C-c0] (fp32, deterministic)."""
    c0 = C if c0 is None else c0
    if not x.is_cuda:
        s = x[:, :C].float().sum(0)
        out0.view(-1).copy_(s[:c0])
        if out1 is not None:
            out1.view(-1).copy_(s[c0:])
        return
    N = _N()
    k = N.kernels()
    assert x.stride(1) == 1 and out0.is_contiguous() and out0.dtype == torch.float32
    parts = k.mbk_colsum_parts(x.shape[0])
    scratch = torch.empty(parts * C, dtype=torch.float32, device=x.device)
    N.check(k.mbk_colsum(x.data_ptr(), int(x.dtype == torch.float32), x.shape[0], C, x.stride(0),
                         scratch.data_ptr(), out0.data_ptr(), c0, N.ptr(out1), N.stream_ptr()),
            "colsum")


def map_gather(segs):
    """segs: [(src fp32 tensor, dst tensor, map int32)]: dst.flat[i] = src.flat[map[i]] or 0."""
    if not segs:
        return
    if not segs[0][1].is_cuda:
        for src, dst, m in segs:
            v = src.reshape(-1)[m.long().clamp(min=0)] * (m >= 0)
            dst.view(-1).copy_(v.reshape(-1))
        return
    N = _N()
    n = len(segs)
    for src, dst, m in segs:
        assert src.dtype == torch.float32 and src.is_contiguous() and dst.is_contiguous()
        assert m.dtype == torch.int32 and m.numel() == dst.numel()
    srcs = (ctypes.c_void_p * n)(*[s.data_ptr() for s, _, _ in segs])
    dsts = (ctypes.c_void_p * n)(*[d.data_ptr() for _, d, _ in segs])
    maps = (ctypes.c_void_p * n)(*[m.data_ptr() for _, _, m in segs])
    ns = (ctypes.c_int * n)(*[d.numel() for _, d, _ in segs])
    bf = (ctypes.c_int * n)(*[int(d.dtype == _BF) for _, d, _ in segs])
    N.check(N.kernels().mbk_map_gather(n, srcs, dsts, maps, ns, bf, N.stream_ptr()), "map_gather")


def value_bwd(dv: torch.Tensor, h: torch.Tensor, w2: torch.Tensor, gw2: torch.Tensor,
              gb2: torch.Tensor, gadd: torch.Tensor | None = None) -> torch.Tensor:
    """Critic output layer v = h . w2 + b2 with h = relu(.): returns dh (bf16, relu mask
    applied) and writes dW2 / db2 (fp32) into gw2 / gb2. gadd: another gradient of the first
    gadd.shape[0] rows of h (fp32 / bf16), added before the relu mask."""
    R, K = h.shape
    if not h.is_cuda:
        dvf = dv.float().reshape(R, 1)
        gw2.view(-1).copy_((dvf * h.float()).sum(0))
        gb2.view(-1).copy_(dvf.sum())
        d = dvf * w2.reshape(1, K)
        if gadd is not None:
            d[:gadd.shape[0]] += gadd.float()
        return (d * (h > 0)).to(_BF)
    N = _N()
    k = N.kernels()
    assert dv.dtype == torch.float32 and dv.is_contiguous() and h.is_contiguous()
    parts = k.mbk_value_bwd_parts(R)
    partial = torch.empty(parts, K + 1, dtype=torch.float32, device=h.device)
    dh = torch.empty(R, K, dtype=_BF, device=h.device)
    if gadd is not None:
        assert gadd.is_contiguous() and gadd.shape[1] == K and gadd.dtype in (torch.float32, _BF)
    N.check(k.mbk_value_bwd(dv.data_ptr(), h.data_ptr(), w2.data_ptr(), R, K, dh.data_ptr(),
                            partial.data_ptr(), N.ptr(gadd),
                            gadd.shape[0] if gadd is not None else 0,
                            int(gadd is not None and gadd.dtype == torch.float32),
                            N.stream_ptr()), "value_bwd")
    colsum(partial, K + 1, gw2, K, gb2)
    return dh


# ============================================================================ weight maps
def _conv_shifts(W: int):
    Wp = W + 2
    return [(ky - 1) * Wp + (kx - 1) for ky in range(3) for kx in range(3)]


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


def conv_maps(cout: int, cin: int):
    """conv3x3 weight [cout, cin, 3, 3]: (fwd B [cout, 9*cp], dgrad B [cp, 9*cout],
    grad map [cout*cin*9] into dW [cout, 9*cp]) index maps (int32, -1 = zero)."""
    cp = _ceil32(cin)
    o = torch.arange(cout).view(-1, 1, 1)
    t = torch.arange(9).view(1, -1, 1)
    c = torch.arange(cp).view(1, 1, -1)
    src = o * cin * 9 + c * 9 + t                                   # [cout, 9, cp]
    fwd = torch.where(c < cin, src, -1).reshape(cout, 9 * cp)
    dgrad = torch.where(c < cin, src, -1).permute(2, 1, 0).reshape(cp, 9 * cout)
    oo = torch.arange(cout).view(-1, 1, 1)
    cc = torch.arange(cin).view(1, -1, 1)
    tt = torch.arange(9).view(1, 1, -1)
    grad = (oo * 9 * cp + tt * cp + cc).reshape(-1)                 # dst (o, c, ky, kx)
    return fwd.int(), dgrad.int(), grad.int()


def convt_maps(cin: int, cout: int):
    """ConvTranspose weight [cin, cout, 3, 3]: per-phase fwd B [cout, ntap*cip] (concatenated),
    dgrad B [cip, 9*cop] (blocks in phase / tap order), grad map [cin*cout*9] into the
    concatenated per-phase dW [cop, ntap*cip]."""
    cip, cop = _ceil32(cin), _ceil32(cout)
    fwd, blocks, where_tap = [], [], {}
    off = 0
    for _, _, taps in _phase_taps(1):
        nt = len(taps)
        o = torch.arange(cout).view(-1, 1, 1)
        c = torch.arange(cip).view(1, 1, -1)
        kk = torch.tensor([ky * 3 + kx for ky, kx, _ in taps]).view(1, -1, 1)
        fwd.append(torch.where(c < cin, c * cout * 9 + o * 9 + kk, -1).reshape(-1))
        for i, (ky, kx, _) in enumerate(taps):
            cc = torch.arange(cip).view(-1, 1)
            oo = torch.arange(cop).view(1, -1)
            blocks.append(torch.where((cc < cin) & (oo < cout), cc * cout * 9 + oo * 9 + ky * 3 + kx,
                                      -1))
            where_tap[ky * 3 + kx] = (off, nt, i)
        off += cop * nt * cip
    dgrad = torch.cat(blocks, dim=1)                                # [cip, 9*cop]
    grad = torch.empty(cin, cout, 9, dtype=torch.int64)
    c = torch.arange(cin).view(-1, 1)
    o = torch.arange(cout).view(1, -1)
    for k, (base, nt, i) in where_tap.items():
        grad[:, :, k] = base + o * (nt * cip) + i * cip + c
    return torch.cat(fwd).int(), dgrad.int(), grad.reshape(-1).int(), off


def critic_maps(k1: int, c: int, hh: int, ww: int):
    """critic Linear(c*hh*ww -> k1), reference NCHW flatten: fwd B [k1, hh*ww*c] (NHWC
    columns), dgrad B [hh*ww*c, k1], grad map [k1*c*hh*ww] from the NHWC-ordered dW."""
    f = c * hh * ww
    k = torch.arange(k1).view(-1, 1, 1, 1)
    y = torch.arange(hh).view(1, -1, 1, 1)
    x = torch.arange(ww).view(1, 1, -1, 1)
    ch = torch.arange(c).view(1, 1, 1, -1)
    src = k * f + ch * hh * ww + y * ww + x                           # [k1, hh, ww, c]
    fwd = src.reshape(k1, -1)
    dgrad = fwd.t().contiguous()
    kk = torch.arange(k1).view(-1, 1, 1, 1)
    cc = torch.arange(c).view(1, -1, 1, 1)
    yy = torch.arange(hh).view(1, 1, -1, 1)
    xx = torch.arange(ww).view(1, 1, 1, -1)
    grad = (kk * f + (yy * ww + xx) * c + cc).reshape(-1)            # dst (k, c, y, x)
    return fwd.int(), dgrad.int(), grad.int()


# ============================================================================ layers
def _pgrad(p) -> torch.Tensor:
    """fp32 buffer a kernel fills with parameter p's gradient (its flat slot when p is a
    direct-gradient parameter, ops/optim.py)."""
    from .optim import grad_out
    return grad_out(p)


def _identity_rm(Hp, Wp):
    """remap writing every row of a padded grid to the same position, zero border"""
    return remap(Hp, Wp, Hp * Wp, Wp, 1, 1, 1, 1, (Hp, Wp), True)


class _EncoderLayer(torch.autograd.Function):
    """conv3x3(+bias) -> relu -> max_pool(3, 2, 1); padded grid in, padded grid out (plus
    the plain pooled map for the critic when ``plain``)."""

    @staticmethod
    def forward(ctx, xp, w, b, wk, wt, gmap, plain):
        ctx.set_materialize_grads(False)
        B, Hp, Wp, cp = xp.shape
        H, W = Hp - 2, Wp - 2
        cout = wk.shape[0]
        y = torch.empty(B, H, W, cout, dtype=_BF, device=xp.device)
        taps_gemm([xp.view(-1, cp)] * 9, _conv_shifts(W), wk, b.detach(), True,
                  out=y.view(-1, cout), rm=remap(Hp, Wp, H * W, W))
        out, pp, idx = pool_fwd(y, plain, True)
        ctx.save_for_backward(xp, pp, idx, wt, gmap)
        ctx.params = (w, b)
        return (pp, out) if plain else pp

    @staticmethod
    def backward(ctx, g_pad, g_plain=None):
        xp, pp, idx, wt, gmap = ctx.saved_tensors
        B, Hp, Wp, cp = xp.shape
        H, W = Hp - 2, Wp - 2
        if g_pad is None and g_plain is None:
            return (None,) * 7
        g1, p1, g2 = (g_pad, 1, g_plain) if g_pad is not None else (g_plain, 0, None)
        dy = pool_bwd(g1.contiguous(), p1, None if g2 is None else g2.contiguous(), 0, pp, 1,
                      idx, H, W)                                      # [B, H+2, W+2, cout]
        cout = dy.shape[-1]
        d2 = dy.view(-1, cout)
        sh = _conv_shifts(W)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(xp)
            taps_gemm([d2] * 9, [-s for s in sh], wt, out=gx.view(-1, cp),
                      rm=_identity_rm(Hp, Wp))
        if ctx.needs_input_grad[1]:
            dw = taps_wgrad(d2, xp.view(-1, cp), sh)                   # [cout, 9*cp]
            gw = _pgrad(ctx.params[0])
            map_gather([(dw, gw, gmap)])
        if ctx.needs_input_grad[2]:
            gb = _pgrad(ctx.params[1])
            colsum(d2, cout, gb)
        return gx, gw, gb, None, None, None, None


class _BitsEncoderLayer(torch.autograd.Function):
    """The first encoder layer (bit-plane input, 32 output channels) on conv.hip's stage-0
    kernels instead of the shifted-row GEMM over the halo'd grid: conv3x3(+bias) with the
    3x3/2 max-pool + argmax in its epilogue (``conv0_row`` on 16-wide maps), relu while
    padding the pooled map into the next layer's grid (grid_gather with itself as the mask);
    backward = relu mask + crop of the next layer's padded dgrad, the argmax max-pool backward
    (``pool_bwd_idx``) and the bit-plane weight-gradient kernel (band layout, bias grad by
    MFMA). No input gradient (the observation). Same maths as ``_EncoderLayer``:
    relu(pool(conv)) == pool(relu(conv)), and the pool argmax only routes gradients where the
    relu passes them."""

    @staticmethod
    def forward(ctx, bits_pad, w, b, enc):
        ctx.set_materialize_grads(False)
        L = enc.layers[0]
        enc.pack_layer(0, w.detach().contiguous())
        n = bits_pad.shape[0]
        Ho, Wo = (L.H + 1) // 2, (L.W + 1) // 2
        pidx = torch.empty(n, Ho, Wo, L.cout, dtype=torch.uint8, device=bits_pad.device)
        p = enc._fwd(L, bits_pad, b.detach(), pool_idx=pidx)         # pooled, pre-relu
        C = L.cout
        pp = grid_gather(p, (0, Ho * Wo * C, Wo * C, C, Ho, Wo, C), p,
                         (0, Ho * Wo * C, Wo * C, C), 1, n, Ho, Wo, C)[0]
        ctx.save_for_backward(bits_pad, p, pidx)
        ctx.enc = enc
        ctx.params = (w, b)
        return pp

    @staticmethod
    def backward(ctx, g_pad):
        bits_pad, p, pidx = ctx.saved_tensors
        enc = ctx.enc
        L = enc.layers[0]
        if g_pad is None or not (ctx.needs_input_grad[1] or ctx.needs_input_grad[2]):
            return (None,) * 4
        n, Ho, Wo, C = p.shape
        k = _N().kernels()
        st = _N().stream_ptr()
        dp = torch.empty_like(p)
        _N().check(k.mbk_crop_relu_mask(g_pad.contiguous().data_ptr(), p.data_ptr(), n, Ho, Wo,
                                        C, dp.data_ptr(), st), "crop_relu_mask")
        dc = torch.empty(n, L.H, L.W, C, dtype=_BF, device=p.device)
        _N().check(k.mbk_pool_bwd_idx(pidx.data_ptr(), dp.data_ptr(), n, L.H, L.W, C,
                                      dc.data_ptr(), st), "pool_bwd_idx")
        gw, gb = _pgrad(ctx.params[0]), _pgrad(ctx.params[1])
        enc._wgrad(L, bits_pad, dc, gw, gb)
        return None, gw, gb, None


class _DecoderLayer(torch.autograd.Function):
    """ConvTranspose2d(k3, s2, p1, op1)(+bias): padded grid in; out = padded grid of the
    relu'd output, or (``crop`` = (h, w)) the final layer's cell-major logits
    [B, h*w*cout] (no relu) cropped to the map."""

    @staticmethod
    def forward(ctx, xp, w, b, bm, bdx, gmap, crop, dw_floats, rows):
        ctx.set_materialize_grads(False)
        B, Hp, Wp, cip = xp.shape
        H, W = Hp - 2, Wp - 2
        cout = w.shape[1]
        B = rows if rows is not None else B      # only the first `rows` images (a prefix)
        x2 = xp.view(-1, cip)[:B * Hp * Wp]
        if crop is None:
            Ho, Wo = 2 * H + 2, 2 * W + 2
            y = torch.empty(B, Ho, Wo, cout, dtype=_BF, device=xp.device)
        else:
            h, wd = crop
            y = torch.empty(B, h * wd * cout, dtype=_BF, device=xp.device)
        y2 = y.view(-1, cout)
        off = 0
        for a, bb, taps in _phase_taps(W):
            nt = len(taps)
            bp = bm[off:off + cout * nt * cip].view(cout, nt * cip)
            off += cout * nt * cip
            if crop is None:
                rm = remap(Hp, Wp, Ho * Wo, Wo, 2, 2, a + 1, bb + 1, (Ho, Wo), True)
            else:
                rm = remap(Hp, Wp, h * wd, wd, 2, 2, a, bb, (h, wd))
            taps_gemm([x2] * nt, [s for _, _, s in taps], bp, b.detach(), crop is None,
                      out=y2, rm=rm)
        ctx.save_for_backward(xp, y if crop is None else None, bdx, gmap)
        ctx.meta = (crop, cout, dw_floats, B)
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, gy):
        xp, y, bdx, gmap = ctx.saved_tensors
        crop, cout, dw_floats, B = ctx.meta
        if gy is None:
            return (None,) * 9
        _, Hp, Wp, cip = xp.shape
        x2 = xp.view(-1, cip)[:B * Hp * Wp]
        H, W = Hp - 2, Wp - 2
        cop = _ceil32(cout)
        gy = gy.contiguous()
        if crop is None:  # padded [B, 2H+2, 2W+2, cout] gradient, relu mask from y
            Wo = 2 * W + 2
            geo = (Wo * cout + cout, (2 * H + 2) * Wo * cout, Wo * cout, cout, 2 * H, 2 * W, cout)
            gps = grid_gather(gy, geo, y, geo[:4], 2, B, H, W, cop)
        else:             # cell-major dlogits [B, h*w*cout]
            h, wd = crop
            geo = (0, h * wd * cout, wd * cout, cout, h, wd, cout)
            gps = grid_gather(gy, geo, None, None, 2, B, H, W, cop)
        phases = _phase_taps(W)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            bases, shifts = [], []
            for p, (_, _, taps) in enumerate(phases):
                for _, _, s in taps:
                    bases.append(gps[p].view(-1, cop))
                    shifts.append(-s)
            gx = torch.empty_like(xp)
            gx2 = gx.view(-1, cip)
            taps_gemm(bases, shifts, bdx, out=gx2[:B * Hp * Wp], rm=_identity_rm(Hp, Wp))
            if B < xp.shape[0]:
                from .copy import zero_
                zero_(gx2[B * Hp * Wp:])
        if ctx.needs_input_grad[1]:
            dw = torch.empty(dw_floats, dtype=torch.float32, device=xp.device)
            off = 0
            for p, (_, _, taps) in enumerate(phases):
                n = cop * len(taps) * cip
                taps_wgrad(gps[p].view(-1, cop), x2, [s for _, _, s in taps],
                           out=dw[off:off + n])
                off += n
            gw = _pgrad(ctx.params[0])
            map_gather([(dw, gw, gmap)])
        if ctx.needs_input_grad[2]:
            gb = _pgrad(ctx.params[1])
            colsum(gps.view(-1, cop), cout, gb)
        return gx, gw, gb, None, None, None, None, None, None


class _Critic(torch.autograd.Function):
    """v = Linear(k1 -> 1)(relu(Linear(F -> k1)(z))) on the plain pooled map z [B, hh, ww, C]
    (NHWC flatten; the first weight's columns are permuted from the reference's NCHW order
    by its index map)."""

    @staticmethod
    def forward(ctx, z, w1, b1, w2, b2, w1p, w1t, w2p, gmap):
        ctx.set_materialize_grads(False)
        B = z.shape[0]
        z2 = z.reshape(B, -1)
        h = gemm_nt(z2, w1p, b1.detach(), relu=True)                # [B, k1] bf16
        v = gemm_nt(h, w2p, b2.detach(), out_dtype=torch.float32)   # [B, 1]
        ctx.save_for_backward(z, h, w1t, gmap, w2)
        ctx.params = (w1, b1, w2, b2)
        return v.view(-1)

    @staticmethod
    def backward(ctx, gv):
        z, h, w1t, gmap, w2 = ctx.saved_tensors
        if gv is None:
            return (None,) * 9
        B = z.shape[0]
        z2 = z.reshape(B, -1)
        k1 = h.shape[1]
        w1, b1, _, b2 = ctx.params
        gw2 = _pgrad(w2)
        gb2 = _pgrad(b2)
        dh = value_bwd(gv.float().contiguous(), h, w2.detach(), gw2, gb2)  # [B, k1] bf16
        gz = gw1 = gb1 = None
        if ctx.needs_input_grad[0]:
            gz = gemm_nt(dh, w1t).view(z.shape)
        if ctx.needs_input_grad[1]:
            dw1 = taps_wgrad(dh, z2, [0])                                 # [k1, F] NHWC cols
            gw1 = _pgrad(w1)
            map_gather([(dw1, gw1, gmap)])
        if ctx.needs_input_grad[2]:
            gb1 = _pgrad(b1)
            colsum(dh, k1, gb1)
        return gz, gw1, gb1, gw2, gb2, None, None, None, None


# ============================================================================ plan
class GridPlan:
    """Index maps of every GridNet weight (built once per model and device) and the
    one-launch weight packing of a forward."""

    def __init__(self, convs, convts, lin1, lin2, zshape, device):
        self.device = device
        self.convs, self.convts, self.lin1, self.lin2 = convs, convts, lin1, lin2
        dev = lambda t: t.to(device)  # noqa: E731
        self.enc = []
        for c in convs:
            fwd, dgrad, grad = conv_maps(c.weight.shape[0], c.weight.shape[1])
            self.enc.append((dev(fwd), dev(dgrad), dev(grad), fwd.shape, dgrad.shape))
        self.dec = []
        for t in convts:
            fwd, dgrad, grad, nfl = convt_maps(t.weight.shape[0], t.weight.shape[1])
            self.dec.append((dev(fwd), dev(dgrad), dev(grad), fwd.shape, dgrad.shape, nfl))
        hh, ww, c = zshape
        # the bit-plane first layer on conv.hip (_BitsEncoderLayer) when it is the 32-plane ->
        # 32-channel conv those kernels implement (CUDA only; the CPU emulation keeps the grid
        # path)
        c0 = convs[0]
        self.enc0 = None
        if (torch.device(device).type == "cuda" and c0.weight.shape[0] == 32
                and c0.weight.shape[1] <= 32 and os.environ.get("MBK_GRID_E1_CONV", "1") == "1"):
            from .encoder import HipEncoder
            self.enc0 = HipEncoder(16 * hh, 16 * ww, c0.weight.shape[1], channels=(32,),
                                   device=device)
        fwd, dgrad, grad = critic_maps(lin1.weight.shape[0], c, hh, ww)
        self.crit = (dev(fwd), dev(dgrad), dev(grad), fwd.shape, dgrad.shape)
        self.w2map = dev(torch.arange(lin2.weight.numel(), dtype=torch.int32))

    def pack(self, with_dgrad: bool):
        """bf16 GEMM operands of every layer (one map_gather launch)."""
        segs, out = [], {"enc": [], "dec": []}

        def seg(p, m, shape):
            t = torch.empty(shape, dtype=_BF, device=self.device)
            segs.append((p.detach(), t, m))
            return t

        for i, (c, (fm, dm, _, fs, ds)) in enumerate(zip(self.convs, self.enc)):
            wk = seg(c.weight, fm, fs)
            wt = seg(c.weight, dm, ds) if with_dgrad and i > 0 else None
            out["enc"].append((wk, wt))
        for t, (fm, dm, _, fs, ds, _) in zip(self.convts, self.dec):
            bm = seg(t.weight, fm, fs)
            bdx = seg(t.weight, dm, ds) if with_dgrad else None
            out["dec"].append((bm, bdx))
        fm, dm, _, fs, ds = self.crit
        out["w1p"] = seg(self.lin1.weight, fm, fs)
        out["w1t"] = seg(self.lin1.weight, dm, ds) if with_dgrad else None
        out["w2p"] = seg(self.lin2.weight, self.w2map, self.lin2.weight.shape)
        map_gather(segs)
        return out


def gridnet_forward(plan: GridPlan, bits: torch.Tensor, h: int, w: int, ph: int, pw: int,
                    n_logits: int | None = None):
    """(logits bf16 [n_logits or n, h*w*78] cell-major, value fp32 [n]) of int32 bit-plane
    obs; with ``n_logits`` the decoder runs on the first n_logits observations only (the
    learner scores T*B of its (T+1)*B rows; the last row only needs its value)."""
    grad = torch.is_grad_enabled()
    pk = plan.pack(grad)
    n = bits.shape[0]
    fast0 = plan.enc0 is not None and bits.is_cuda
    if fast0:
        bp = torch.empty(n, ph * pw, dtype=torch.int32, device=bits.device)
        _N().check(_N().kernels().mbk_bits_pad(bits.reshape(n, h * w).contiguous().data_ptr(),
                                               n, h, w, ph, pw, bp.data_ptr(), _N().stream_ptr()),
                   "bits_pad")
    else:
        x = bits_grid(bits.reshape(n, h * w).contiguous(), h, w, ph + 2, pw + 2)
    z = None
    nl = len(plan.convs)
    for i, (c, (wk, wt), (_, _, gm, _, _)) in enumerate(zip(plan.convs, pk["enc"], plan.enc)):
        if i == 0 and fast0 and nl > 1:
            x = _BitsEncoderLayer.apply(bp, c.weight, c.bias, plan.enc0)
        elif i == nl - 1:
            x, z = _EncoderLayer.apply(x, c.weight, c.bias, wk, wt, gm, True)
        else:
            x = _EncoderLayer.apply(x, c.weight, c.bias, wk, wt, gm, False)
    y = x
    nd = len(plan.convts)
    for j, (t, (bm, bdx), (_, _, gm, _, _, nfl)) in enumerate(zip(plan.convts, pk["dec"],
                                                                  plan.dec)):
        crop = (h, w) if j == nd - 1 else None
        y = _DecoderLayer.apply(y, t.weight, t.bias, bm, bdx, gm, crop, nfl,
                                n_logits if j == 0 else None)
    v = _Critic.apply(z, plan.lin1.weight, plan.lin1.bias, plan.lin2.weight, plan.lin2.bias,
                      pk["w1p"], pk["w1t"], pk["w2p"], plan.crit[2])
    return y, v
