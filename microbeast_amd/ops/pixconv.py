"""GridNet on the pixel-major "PBC" layout ([pixel][image][channel], bf16), csrc/kernels/pixconv.hip.

GridNet (BASELINE config 2, ``models/gridnet.py``) runs conv3x3 + relu + max-pool(3, 2, 1)
encoder layers from the map down to 1x1, stride-2 transposed convs (k3 s2 p1 op1) back up and
a two-layer critic on the 1x1 code. With images inside pixels every layer is, per OUTPUT
pixel P, one GEMM over images:

    out[P] = bias + sum_{(q, t) in pairs(P)} A[q] . W_t^T         (``pconv``)

where pairs(P) lists only the in-range (source pixel, tap) pairs: 4..9 for a conv3x3, 1/2/4
for a transposed conv (its sub-pixel phases), and the z pixels for the critic's first Linear.
The input gradient is the same kernel over the inverse pair lists with transposed weights; the
weight gradient (``pwgrad``) is a split-K GEMM over (pair, image) rows reduced straight into
the parameter's layout (``reduce_map``). Pooling keeps a uint8 argmax and its backward is a
gather (``ppool_bwd``) that also applies the relu-after-pool mask.

Compared with the padded-grid shifted-row GEMMs this replaces (``ops/gridconv.py`` up to
round 3), no MFMA work is spent on halo rows (1.6x..9x the useful work on the 8x8..1x1 grids),
the decoder needs no phase-gather pass, and the first layer's NHWC output (conv.hip stage-0
kernels) is consumed in place through the (pixel stride, image stride) operand addressing.

Two specialisations sit on top:

* the 8x8 32 -> 64 conv runs on whole-image LDS tiles (``imgconv`` forward / input gradient,
  ``imgwgrad``): all 9 taps read the input from LDS instead of re-reading it through L2;
* the logits layer runs on the active cells only (``Cells``: compacted (cell, sample) rows;
  ``pconv(cells=...)`` forward over them, compact masked-cell kernels in ``cell_head``,
  ``pwgrad(cells=...)`` and the sparse input gradient ``pconv(gather=...)``).

Every launcher has a plain-torch emulation of the same index maths (CPU tensors), so the whole
network is unit-tested on CPU against the nn.Module (tests/test_pixconv.py); the GPU tests run
the kernels against the emulation / fp32.
"""
from __future__ import annotations

import ctypes

import torch

_BF = torch.bfloat16
LOGIT_LD = 96     # row stride of the pixel-major logits (78 + zero padding, K % 32 == 0)
_MAXP = 16        # pconv pairs per output pixel (kernel limit)


def _ceil32(c: int) -> int:
    return -(-c // 32) * 32


def _N():
    from .. import _native as N
    return N



# ---- CPU emulation hook -----------------------------------------------------------------
# The pixel-major kernels run on the GPU only. Their plain-torch emulation on CPU tensors (the
# same bf16 maths, per-pixel loops: an oracle, not a product path) lives in the test suite
# (tests/pixconv_emulation.py) and is registered by it; GridNetAgent.emulate routes a CPU model
# through it.
_EMULATION = None


def set_emulation(module) -> None:
    """Register the CPU emulation of this module's kernels (tests/pixconv_emulation.py)."""
    global _EMULATION
    _EMULATION = module


def _emulation():
    if _EMULATION is None:
        raise RuntimeError("pixel-major GridNet kernels need a GPU: their CPU emulation is test "
                           "code (tests/pixconv_emulation.py, pixconv.set_emulation)")
    return _EMULATION


def _view(t: torch.Tensor, ps: int, bs: int, rows: int, cols: int, P: int) -> torch.Tensor:
    """rows x cols strided view at pixel P of a (pixel stride, image stride) operand"""
    return torch.as_strided(t.reshape(-1), (rows, cols), (bs, 1), P * ps)


# ============================================================================ tables
def conv_pairs(H: int, W: int):
    """stride-1 3x3 pad-1 conv on H x W: (fwd [(P, [(q, t)])], dgrad [(q, [(P, t)])],
    wgrad per tap [[(P, q)]])."""
    fwd, dg, wg = [], [[] for _ in range(H * W)], [[] for _ in range(9)]
    for y in range(H):
        for x in range(W):
            P, ents = y * W + x, []
            for ky in range(3):
                for kx in range(3):
                    yy, xx = y + ky - 1, x + kx - 1
                    if 0 <= yy < H and 0 <= xx < W:
                        q, t = yy * W + xx, ky * 3 + kx
                        ents.append((q, t))
                        dg[q].append((P, t))
                        wg[t].append((P, q))
            fwd.append((P, ents))
    return fwd, [(q, e) for q, e in enumerate(dg)], wg


def convt_pairs(H: int, W: int, crop=None):
    """ConvTranspose2d(k3, s2, p1, op1) H x W -> 2H x 2W, output cropped to ``crop`` = (h, w)
    (output pixel index Y * w + X): out(Y) gets in(iy) . w[ky] for Y = 2 iy - 1 + ky."""
    Ho, Wo = crop if crop is not None else (2 * H, 2 * W)
    fwd, dg, wg = [], [[] for _ in range(H * W)], [[] for _ in range(9)]
    for Y in range(Ho):
        for X in range(Wo):
            P, ents = Y * Wo + X, []
            for ky in range(3):
                iy2 = Y + 1 - ky
                if iy2 % 2 or not 0 <= iy2 // 2 < H:
                    continue
                for kx in range(3):
                    ix2 = X + 1 - kx
                    if ix2 % 2 or not 0 <= ix2 // 2 < W:
                        continue
                    q, t = (iy2 // 2) * W + ix2 // 2, ky * 3 + kx
                    ents.append((q, t))
                    dg[q].append((P, t))
                    wg[t].append((P, q))
            fwd.append((P, ents))
    return fwd, [(q, e) for q, e in enumerate(dg)], wg


def critic_pairs(npix: int):
    """critic Linear over the z pixels as one output 'pixel' with a tap per z pixel"""
    return ([(0, [(P, P) for P in range(npix)])], [(P, [(0, P)]) for P in range(npix)],
            [[(0, P)] for P in range(npix)])


class Tab:
    """A device pair table plus the host-side index bounds the launchers check operand sizes
    against before a kernel runs (an out-of-range pixel would read / write outside a buffer)."""

    def __init__(self, t: torch.Tensor, src_max: int, tap_max: int, dst_max: int):
        self.t, self.src_max, self.tap_max, self.dst_max = t, src_max, tap_max, dst_max

    @property
    def shape(self):
        return self.t.shape


def pconv_table(rows, device) -> Tab:
    """int32 [nz, 2 + maxp]: P_out, count, (q << 8 | t)... (rows with no pair are kept: their
    output is bias only)"""
    w = max(1, max(len(e) for _, e in rows))
    assert w <= _MAXP, f"{w} pairs per output pixel > {_MAXP}"
    tab = torch.zeros(len(rows), 2 + w, dtype=torch.int32)
    qm = tm = 0
    for z, (P, ents) in enumerate(rows):
        tab[z, 0], tab[z, 1] = P, len(ents)
        for j, (q, t) in enumerate(ents):
            assert q < (1 << 23) and t < 256
            tab[z, 2 + j] = (q << 8) | t
            qm, tm = max(qm, q), max(tm, t)
    return Tab(tab.to(device), qm, tm, max(P for P, _ in rows))


def wgrad_table(taps, device) -> Tab:
    """int32 [ntap, 1 + maxc]: count, (P << 16 | q)..."""
    w = max(1, max(len(e) for e in taps))
    tab = torch.zeros(len(taps), 1 + w, dtype=torch.int32)
    qm = pm = 0
    for t, ents in enumerate(taps):
        tab[t, 0] = len(ents)
        for j, (P, q) in enumerate(ents):
            assert P < (1 << 15) and q < (1 << 16)
            tab[t, 1 + j] = (P << 16) | q
            qm, pm = max(qm, q), max(pm, P)
    return Tab(tab.to(device), qm, len(taps) - 1, pm)


def _fits(t: torch.Tensor, last_pix: int, ps: int, rows: int, bs: int, cols: int, what: str):
    end = last_pix * ps + (rows - 1) * bs + cols
    assert end <= t.numel(), f"{what}: operand too small ({end} > {t.numel()} elements)"


# ============================================================================ launchers
def pconv(A, a_ps, a_bs, cin, B, tab, N, M, C, c_ps, c_bs, bias=None, relu=False, a_relu=False,
          mask=None, cells=None, gather=None):
    """C[P][b][:N] = relu?(bias + sum_{(q, t)} relu?(A[q][b][:cin]) . B[t][:N][:cin]^T) for
    every table row (P = its output pixel), b < M; masked to 0 where mask (C's layout) <= 0.
    Operands are addressed as (pixel stride, image stride) in elements; B is [ntap][N][cin].

    cells (``Cells``, sparse rows): table row P computes only the compact rows of cell bucket P
    (images cells.rowimg), written to C's compact rows (image stride c_bs; c_ps unused).
    gather (``Cells``): A row of pair source P and image b is compact row cellrow[P][b] of A
    (image stride a_bs; a_ps unused), zero when the cell is inactive."""
    assert (tab.tap_max + 1) * N * cin <= B.numel(), "pconv B too small"
    if cells is not None:
        _fits(A, tab.src_max, a_ps, M, a_bs, cin, "pconv A")
        assert cells.cap * c_bs <= C.numel() and tab.shape[0] == cells.S and mask is None
    elif gather is not None:
        assert gather.cap * a_bs <= A.numel() and tab.src_max < gather.S and M == gather.n
        _fits(C, tab.dst_max, c_ps, M, c_bs, N, "pconv C")
    else:
        _fits(A, tab.src_max, a_ps, M, a_bs, cin, "pconv A")
        _fits(C, tab.dst_max, c_ps, M, c_bs, N, "pconv C")
    if mask is not None:
        _fits(mask, tab.dst_max, c_ps, M, c_bs, N, "pconv mask")
    if not C.is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().pconv(**locals())
    N_ = _N()
    for t in (A, B, C, mask):
        assert t is None or (t.dtype == _BF and t.is_contiguous())
    assert bias is None or (bias.dtype == torch.float32 and bias.is_contiguous())
    assert tab.t.dtype == torch.int32 and tab.t.is_cuda
    mode, sp = (1, cells) if cells is not None else ((2, gather) if gather is not None else (0, None))
    args = (ctypes.c_longlong * 26)(
        A.data_ptr(), a_ps, a_bs, cin, int(a_relu), B.data_ptr(), tab.t.data_ptr(), tab.shape[1],
        tab.shape[0], bias.data_ptr() if bias is not None else 0, int(relu), C.data_ptr(), c_ps,
        c_bs, mask.data_ptr() if mask is not None else 0, M, N, mode,
        sp.bucket_off.data_ptr() if mode == 1 else 0, sp.bucket_cnt.data_ptr() if mode == 1 else 0,
        sp.tile_off.data_ptr() if mode == 1 else 0, sp.totals.data_ptr() if mode == 1 else 0,
        sp.rowimg.data_ptr() if mode == 1 else 0, sp.S if mode == 1 else 0,
        sp.cellrow.data_ptr() if mode == 2 else 0,
        2048 if mode == 1 else tab.tap_max + 1)   # mode 1: persistent grid; 2: taps of B
    N_.check(N_.kernels().mbk_pconv(args, N_.stream_ptr()), "pconv")
    return C



class Cells:
    """The active cells (any legal action) of n samples x S map cells, compacted into rows in
    (cell, sample) order and bucketed by cell: the sparse logits layer computes, scores and
    back-propagates only these rows (``pixconv.hip`` cells_* kernels; torch on CPU).

    rowimg / rowcell [cap]: sample and cell index (sample * S + cell) of each compact row;
    cellrow [S * n]: compact row of (cell, sample) or -1; bucket_off / bucket_cnt [S],
    tile_off [S + 1] (128-row tiles); totals = [rows, tiles] (device ints: nothing syncs)."""

    TM = 128

    def __init__(self, mask_bits: torch.Tensor, n: int, S: int):
        self.n, self.S, self.cap = n, S, n * S
        dev = mask_bits.device
        m = mask_bits.reshape(n, S, 3)
        if dev.type != "cuda":
            act = (m != 0).any(-1)                       # [n, S]
            pm = act.t().contiguous()                    # [S, n]
            idx = pm.nonzero()                           # (P, b) sorted by P then b
            P, b = idx[:, 0].int(), idx[:, 1].int()
            nact = idx.shape[0]
            self.rowimg = torch.zeros(self.cap, dtype=torch.int32)
            self.rowcell = torch.zeros(self.cap, dtype=torch.int32)
            self.rowimg[:nact] = b
            self.rowcell[:nact] = b * S + P
            self.bucket_cnt = pm.sum(1).int()
            self.bucket_off = (torch.cumsum(self.bucket_cnt, 0) - self.bucket_cnt).int()
            tiles = (self.bucket_cnt + self.TM - 1) // self.TM
            self.tile_off = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(tiles, 0)]).int()
            self.cellrow = torch.full((S * n,), -1, dtype=torch.int32)
            self.cellrow[(P.long() * n + b.long())] = torch.arange(nact, dtype=torch.int32)
            self.totals = torch.tensor([nact, int(self.tile_off[-1])], dtype=torch.int32)
            return
        N_ = _N()
        k = N_.kernels()
        assert mask_bits.dtype == torch.int32 and mask_bits.is_contiguous()
        nchunk = k.mbk_cells_nchunk(n)
        i32 = dict(dtype=torch.int32, device=dev)
        counts = torch.empty(S * nchunk, **i32)
        offs = torch.empty(S * nchunk, **i32)
        self.bucket_off = torch.empty(S, **i32)
        self.bucket_cnt = torch.empty(S, **i32)
        self.tile_off = torch.empty(S + 1, **i32)
        self.totals = torch.empty(2, **i32)
        self.rowimg = torch.empty(self.cap, **i32)
        self.rowcell = torch.empty(self.cap, **i32)
        self.cellrow = torch.empty(S * n, **i32)
        N_.check(k.mbk_cells_compact(mask_bits.data_ptr(), n, S, self.TM, counts.data_ptr(),
                                     offs.data_ptr(), self.bucket_off.data_ptr(),
                                     self.bucket_cnt.data_ptr(), self.tile_off.data_ptr(),
                                     self.totals.data_ptr(), self.rowimg.data_ptr(),
                                     self.rowcell.data_ptr(), self.cellrow.data_ptr(),
                                     N_.stream_ptr()), "cells_compact")

    def rows_colsum(self, Z: torch.Tensor, ld: int, C: int, out: torch.Tensor):
        """out[:C] = column sums of the compact rows of Z [cap][ld] (fp32, fixed order)"""
        if not Z.is_cuda:  # CPU: the test suite's emulation (set_emulation)
            return _emulation().rows_colsum(**locals())
        N_ = _N()
        k = N_.kernels()
        nblk = 256
        partial = torch.empty(nblk * C, dtype=torch.float32, device=Z.device)
        N_.check(k.mbk_rows_colsum(Z.data_ptr(), ld, C, self.totals.data_ptr(), nblk,
                                   partial.data_ptr(), N_.stream_ptr()), "rows_colsum")
        ident = _ident_map(C, Z.device)
        N_.check(k.mbk_reduce_map(partial.data_ptr(), nblk, C, ident.data_ptr(), C,
                                  out.data_ptr(), N_.stream_ptr()), "reduce_map")


_IDENT = {}


def _ident_map(C: int, device) -> torch.Tensor:
    key = (C, str(device))
    if key not in _IDENT:
        _IDENT[key] = torch.arange(C, dtype=torch.int32, device=device)
    return _IDENT[key]


def imgconv(A, a_ps, a_bs, cin, B, N, M, C, c_ps, c_bs, H, bias=None, relu=False, a_relu=False,
            mask=None):
    """conv3x3 / pad 1 on H x H maps with whole images in LDS (``imgconv_kernel``; GPU only):
    C[P][b][:N] = relu?(bias + sum_t relu?(A[P + s_t][b]) . B[t]^T), B [9][N][cin] in tap order
    (ky, kx) with source offset (ky - 1, kx - 1); (pixel stride, image stride) operands."""
    assert A.is_cuda and 9 * N * cin <= B.numel()
    _fits(A, H * H - 1, a_ps, M, a_bs, cin, "imgconv A")
    _fits(C, H * H - 1, c_ps, M, c_bs, N, "imgconv C")
    if mask is not None:
        _fits(mask, H * H - 1, c_ps, M, c_bs, N, "imgconv mask")
    N_ = _N()
    args = (ctypes.c_longlong * 17)(A.data_ptr(), a_ps, a_bs, cin, int(a_relu), B.data_ptr(), 0,
                                    0, 0, bias.data_ptr() if bias is not None else 0, int(relu),
                                    C.data_ptr(), c_ps, c_bs,
                                    mask.data_ptr() if mask is not None else 0, M, N)
    N_.check(N_.kernels().mbk_imgconv(args, H, N_.stream_ptr()), "imgconv")
    return C


_BIAS_MAPS: dict = {}
_INV_MAPS: dict = {}


def _reduce_to(k, N_, partial, parts: int, stride: int, gmap: torch.Tensor, out: torch.Tensor,
               nw: int | None = None, bias_out: torch.Tensor | None = None):
    """out.flat[j] = sum_p partial[p, gmap[j]] (0 where gmap[j] < 0): walked in partial order
    through the inverse map (``reduce_inv_kernel``: coalesced reads) when gmap is injective,
    else the gather form (``reduce_map_kernel``). The inverse is built once per map. With
    ``bias_out``, partial entries [nw, stride) are the bias sums: bias_out = their totals."""
    nw = stride if nw is None else nw
    if bias_out is not None:
        assert bias_out.dtype == torch.float32 and bias_out.numel() == stride - nw
    key = (gmap.data_ptr(), gmap.numel(), nw)
    ent = _INV_MAPS.get(key)
    if ent is None:
        g = gmap.long()
        valid = g >= 0
        src = g[valid]
        inv = None
        if src.numel() == 0 or (int(src.max()) < nw and
                                torch.unique(src).numel() == src.numel()):
            inv = torch.full((nw,), -1, dtype=torch.int32, device=gmap.device)
            inv[src] = torch.nonzero(valid).squeeze(1).to(torch.int32)
        ent = _INV_MAPS[key] = (inv, bool(valid.all()), gmap)   # gmap kept alive with its key
    inv, full, _ = ent
    if inv is None:
        N_.check(k.mbk_reduce_map(partial.data_ptr(), parts, stride, gmap.data_ptr(), out.numel(),
                                  out.data_ptr(), N_.stream_ptr()), "reduce_map")
        if bias_out is not None:
            N_.check(k.mbk_reduce_map(partial.data_ptr(), parts, stride,
                                      _bias_map(stride - nw, nw, out.device).data_ptr(),
                                      stride - nw, bias_out.data_ptr(), N_.stream_ptr()),
                     "reduce_map bias")
        return
    if not full:
        N_.check(k.mbk_memset(out.data_ptr(), 0, out.numel() * 4, N_.stream_ptr()), "memset")
    nm = stride if bias_out is not None else nw
    N_.check(k.mbk_reduce_inv(partial.data_ptr(), parts, stride, inv.data_ptr(), nm,
                              out.data_ptr(), bias_out.data_ptr() if bias_out is not None else 0,
                              nw, N_.stream_ptr()), "reduce_inv")


def imgwgrad(g, g_ps, g_bs, O, x, x_ps, x_bs, I, M, gmap, out, H, x_relu=False, bias_out=None):
    """``pwgrad`` of a full conv3x3 on H x H maps with whole images in LDS
    (``imgwgrad_kernel``; GPU only): dW [9][O][I] -> out via gmap. The kernel also sums dy
    per output channel (an all-ones MFMA column); ``bias_out`` receives that bias gradient."""
    assert g.is_cuda and out.is_cuda
    _fits(g, H * H - 1, g_ps, M, g_bs, O, "imgwgrad g")
    _fits(x, H * H - 1, x_ps, M, x_bs, I, "imgwgrad x")
    N_ = _N()
    k = N_.kernels()
    parts = k.mbk_imgwgrad_parts()
    stride = 9 * O * I + O
    partial = torch.empty(parts * stride, dtype=torch.float32, device=out.device)
    args = (ctypes.c_longlong * 15)(g.data_ptr(), g_ps, g_bs, O, x.data_ptr(), x_ps, x_bs, I,
                                    int(x_relu), 0, 0, 9, M, parts, partial.data_ptr())
    N_.check(k.mbk_imgwgrad(args, H, N_.stream_ptr()), "imgwgrad")
    _reduce_to(k, N_, partial, parts, stride, gmap, out, 9 * O * I, bias_out)
    return out




def _imgconv_ok(L, dev) -> bool:
    """the image-tile kernel covers GridNet's 8x8 32 -> 64 conv (forward and input gradient)"""
    return (dev.type == "cuda" and L.H == 8 and L.W == 8 and L.cin == 32
            and L.cout == 64)


def pwgrad(g, g_ps, g_bs, O, x, x_ps, x_bs, I, tab, M, gmap, out, x_relu=False, cells=None):
    """out.flat[j] = dW[gmap[j]] (0 where gmap < 0), dW [ntap][O][I] fp32 with
    dW[t] = sum_{(P, q) in tab[t]} sum_{b < M} g[P][b][:O]^T relu?(x[q][b][:I]).
    cells: g holds compact rows (image stride g_bs) and pair (P, q) runs over cell bucket P's
    rows, x rows gathered by their images."""
    ntap = tab.shape[0]
    if cells is None:
        _fits(g, tab.dst_max, g_ps, M, g_bs, O, "pwgrad g")
    else:
        assert cells.cap * g_bs <= g.numel() and tab.dst_max < cells.S and M == cells.n
    _fits(x, tab.src_max, x_ps, M, x_bs, I, "pwgrad x")
    if not out.is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().pwgrad(**locals())
    N_ = _N()
    k = N_.kernels()
    assert g.dtype == _BF and x.dtype == _BF and g.is_contiguous() and x.is_contiguous()
    assert out.is_contiguous() and out.dtype == torch.float32 and gmap.numel() == out.numel()
    # rows mode: fine row ranges (the buckets are small and uneven; empty ranges exit at once)
    parts = min(512, max(1, -(-M // 1024))) if cells is not None else k.mbk_pwgrad_parts(M, O, I, ntap)
    stride = ntap * O * I
    partial = torch.empty(parts * stride, dtype=torch.float32, device=out.device)
    args = (ctypes.c_longlong * 18)(g.data_ptr(), g_ps, g_bs, O, x.data_ptr(), x_ps, x_bs, I,
                                    int(x_relu), tab.t.data_ptr(), tab.shape[1], ntap, M, parts,
                                    partial.data_ptr(),
                                    cells.bucket_off.data_ptr() if cells is not None else 0,
                                    cells.bucket_cnt.data_ptr() if cells is not None else 0,
                                    cells.rowimg.data_ptr() if cells is not None else 0)
    N_.check(k.mbk_pwgrad(args, N_.stream_ptr()), "pwgrad")
    _reduce_to(k, N_, partial, parts, stride, gmap, out)
    return out


def _bias_map(O: int, off: int, device) -> torch.Tensor:
    key = (O, off, str(device))
    m = _BIAS_MAPS.get(key)
    if m is None:
        m = _BIAS_MAPS[key] = (torch.arange(O, dtype=torch.int32) + off).to(device)
    return m


def pwgrad_all(g, g_ps, g_bs, O, x, x_ps, x_bs, I, ftab, ntap, M, gmap, out, x_relu=False,
               bias_out=None):
    """``pwgrad`` over the forward pair table (per output pixel P: its (q, t) pairs): g[P] is
    read once per 64-image stage for every tap of P (``pwgrad_all_kernel``); ntap <= 9.
    ``bias_out`` (fp32 [O]) receives sum over the table's output pixels and images of g."""
    assert ntap <= 9 and ftab.tap_max < ntap
    _fits(g, ftab.dst_max, g_ps, M, g_bs, O, "pwgrad_all g")
    _fits(x, ftab.src_max, x_ps, M, x_bs, I, "pwgrad_all x")
    if not out.is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().pwgrad_all(**locals())
    N_ = _N()
    k = N_.kernels()
    assert g.dtype == _BF and x.dtype == _BF and g.is_contiguous() and x.is_contiguous()
    assert out.is_contiguous() and out.dtype == torch.float32 and gmap.numel() == out.numel()
    parts = k.mbk_pwgrad_all_parts(M, O, I)
    stride = ntap * O * I + O
    partial = torch.empty(parts * stride, dtype=torch.float32, device=out.device)
    args = (ctypes.c_longlong * 16)(g.data_ptr(), g_ps, g_bs, O, x.data_ptr(), x_ps, x_bs, I,
                                    int(x_relu), ftab.t.data_ptr(), ftab.shape[1], ftab.shape[0],
                                    ntap, M, parts, partial.data_ptr())
    N_.check(k.mbk_pwgrad_all(args, N_.stream_ptr()), "pwgrad_all")
    _reduce_to(k, N_, partial, parts, stride, gmap, out, ntap * O * I, bias_out)
    return out


def _wgrad(g, g_ps, g_bs, O, x, x_ps, x_bs, I, L, ntap, M, out, x_relu=False, bias_out=None):
    """weight gradient of a dense layer: the all-taps form for the 3x3 convs (~7.6 pairs per
    output pixel share one staged g row; it also yields the bias gradient), the per-tap form
    for the transposed convs and the critic (1-4 pairs per output pixel: nothing to share,
    measured 2x slower all-taps). ``bias_out`` (with g as [pixels][M][O] rows): sum of g."""
    if ntap <= 9 and L.mean_pairs >= 4.0:
        return pwgrad_all(g, g_ps, g_bs, O, x, x_ps, x_bs, I, L.tf, ntap, M, L.gmap, out,
                          x_relu=x_relu, bias_out=bias_out)
    if bias_out is not None:
        colsum(g.view(-1, O), O, bias_out)
    return pwgrad(g, g_ps, g_bs, O, x, x_ps, x_bs, I, L.tw, M, L.gmap, out, x_relu=x_relu)


def ppool_fwd(y, H: int, W: int, n: int, C: int):
    """max_pool(3, 2, 1) of y [H*W][n][C] -> (pooled [Ho*Wo][n][C], idx uint8 = ky*3+kx of
    the first maximum in scan order)"""
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    out = torch.empty(Ho * Wo, n, C, dtype=_BF, device=y.device)
    idx = torch.empty(Ho * Wo, n, C, dtype=torch.uint8, device=y.device)
    if not y.is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().ppool_fwd(**locals())
    N_ = _N()
    assert y.is_contiguous() and y.dtype == _BF and C % 8 == 0
    N_.check(N_.kernels().mbk_ppool_fwd(y.data_ptr(), H, W, n, C, out.data_ptr(), idx.data_ptr(),
                                        N_.stream_ptr()), "ppool_fwd")
    return out, idx


def ppool_bwd(g1, n1: int, g2, n2: int, pooled, idx, H: int, W: int, n: int, C: int):
    """gradient of relu(max_pool(conv)) w.r.t. conv [H*W][n][C]: g1 [Po][n1][C] (+ g2
    [Po][n2][C]) routed to the argmax where pooled > 0."""
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    if not pooled.is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().ppool_bwd(**locals())
    N_ = _N()
    for t in (g1, g2, pooled):
        assert t is None or (t.is_contiguous() and t.dtype == _BF)
    dy = torch.empty(H * W, n, C, dtype=_BF, device=pooled.device)
    N_.check(N_.kernels().mbk_ppool_bwd(g1.data_ptr(), n1 * C, n1, N_.ptr(g2), n2 * C, n2,
                                        pooled.data_ptr(), idx.data_ptr(), H, W, n, C,
                                        dy.data_ptr(), N_.stream_ptr()), "ppool_bwd")
    return dy


def colsum(x: torch.Tensor, C: int, out: torch.Tensor, c0: int | None = None,
           out1: torch.Tensor | None = None):
    """Column sums of the first C columns of 2-D x into out[:c0] and out1[:C-c0] (fp32,
    deterministic)."""
    c0 = C if c0 is None else c0
    if not x.is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().colsum(**locals())
    N_ = _N()
    k = N_.kernels()
    assert x.stride(1) == 1 and out.is_contiguous() and out.dtype == torch.float32
    parts = k.mbk_colsum_parts(x.shape[0])
    scratch = torch.empty(parts * C, dtype=torch.float32, device=x.device)
    N_.check(k.mbk_colsum(x.data_ptr(), int(x.dtype == torch.float32), x.shape[0], C, x.stride(0),
                          scratch.data_ptr(), out.data_ptr(), c0, N_.ptr(out1), N_.stream_ptr()),
             "colsum")


def map_gather(segs):
    """segs: [(src fp32 tensor, dst tensor, map int32)]: dst.flat[i] = src.flat[map[i]] or 0."""
    if not segs:
        return
    if not segs[0][1].is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().map_gather(**locals())
    N_ = _N()
    n = len(segs)
    for src, dst, m in segs:
        assert src.dtype == torch.float32 and src.is_contiguous() and dst.is_contiguous()
        assert m.dtype == torch.int32 and m.numel() == dst.numel()
    srcs = (ctypes.c_void_p * n)(*[s.data_ptr() for s, _, _ in segs])
    dsts = (ctypes.c_void_p * n)(*[d.data_ptr() for _, d, _ in segs])
    maps = (ctypes.c_void_p * n)(*[m.data_ptr() for _, _, m in segs])
    ns = (ctypes.c_int * n)(*[d.numel() for _, d, _ in segs])
    bf = (ctypes.c_int * n)(*[int(d.dtype == _BF) for _, d, _ in segs])
    N_.check(N_.kernels().mbk_map_gather(n, srcs, dsts, maps, ns, bf, N_.stream_ptr()),
             "map_gather")


def gemm_nt(a, b, bias=None, out_dtype=None):
    """a . b^T + bias on gemm.hip: a [M, K], b [N, K] bf16, K % 8 == 0."""
    out_dtype = out_dtype or _BF
    if not a.is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().gemm_nt(**locals())
    N_ = _N()
    assert a.is_contiguous() and b.is_contiguous() and a.dtype == _BF and b.dtype == _BF
    out = torch.empty(a.shape[0], b.shape[0], dtype=out_dtype, device=a.device)
    N_.check(N_.kernels().mbk_gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), N_.ptr(bias),
                                      a.shape[0], b.shape[0], a.shape[1], a.shape[1], b.shape[1],
                                      b.shape[0], 0, int(out_dtype == _BF), 0, N_.stream_ptr()),
             "gemm_nt")
    return out


def value_bwd(dv: torch.Tensor, h: torch.Tensor, w2: torch.Tensor, gw2: torch.Tensor,
              gb2: torch.Tensor, gadd: torch.Tensor | None = None) -> torch.Tensor:
    """Critic output layer v = h . w2 + b2 with h = relu(.): returns dh (bf16, relu mask
    applied) and writes dW2 / db2 (fp32) into gw2 / gb2. gadd: another gradient of the first
    gadd.shape[0] rows of h (fp32 / bf16), added before the relu mask."""
    R, K = h.shape
    if not h.is_cuda:  # CPU: the test suite's emulation (set_emulation)
        return _emulation().value_bwd(**locals())
    N_ = _N()
    k = N_.kernels()
    assert dv.dtype == torch.float32 and dv.is_contiguous() and h.is_contiguous()
    parts = k.mbk_value_bwd_parts(R)
    partial = torch.empty(parts, K + 1, dtype=torch.float32, device=h.device)
    dh = torch.empty(R, K, dtype=_BF, device=h.device)
    if gadd is not None:
        assert gadd.is_contiguous() and gadd.shape[1] == K and gadd.dtype in (torch.float32, _BF)
    N_.check(k.mbk_value_bwd(dv.data_ptr(), h.data_ptr(), w2.data_ptr(), R, K, dh.data_ptr(),
                             partial.data_ptr(), N_.ptr(gadd),
                             gadd.shape[0] if gadd is not None else 0,
                             int(gadd is not None and gadd.dtype == torch.float32),
                             N_.stream_ptr()), "value_bwd")
    colsum(partial, K + 1, gw2, K, gb2)   # dW2 = columns 0..K-1, db2 = column K
    return dh


# ============================================================================ weight maps
def conv_maps(cout: int, cin: int):
    """Conv2d weight [cout, cin, 3, 3] (flat index o*cin*9 + c*9 + t): fwd B [9][cout][cin],
    dgrad B [9][cin][cout_p] (zero rows / cols past the real counts), and the gradient map
    param (o, c, t) -> dW [9][cout][cin] (the pwgrad output with O = cout, I = cin)."""
    t = torch.arange(9).view(9, 1, 1)
    o = torch.arange(cout).view(1, -1, 1)
    c = torch.arange(cin).view(1, 1, -1)
    fwd = (o * cin * 9 + c * 9 + t).reshape(-1)
    cop = _ceil32(cout)
    c2 = torch.arange(cin).view(1, -1, 1)
    o2 = torch.arange(cop).view(1, 1, -1)
    dg = torch.where(o2 < cout, o2 * cin * 9 + c2 * 9 + t, -1).reshape(-1)
    oo = torch.arange(cout).view(-1, 1, 1)
    cc = torch.arange(cin).view(1, -1, 1)
    tt = torch.arange(9).view(1, 1, -1)
    grad = (tt * cout * cin + oo * cin + cc).reshape(-1)
    return fwd.int(), dg.int(), grad.int(), cop


def convt_maps(cin: int, cout: int, gO: int):
    """ConvTranspose2d weight [cin, cout, 3, 3] (flat c*cout*9 + o*9 + t): fwd B
    [9][cout][cin], dgrad B [9][cin][gO] (gO >= cout: the gradient operand's channel count),
    gradient map param (c, o, t) -> dW [9][gO][cin]."""
    t = torch.arange(9).view(9, 1, 1)
    o = torch.arange(cout).view(1, -1, 1)
    c = torch.arange(cin).view(1, 1, -1)
    fwd = (c * cout * 9 + o * 9 + t).reshape(-1)
    c2 = torch.arange(cin).view(1, -1, 1)
    o2 = torch.arange(gO).view(1, 1, -1)
    dg = torch.where(o2 < cout, c2 * cout * 9 + o2 * 9 + t, -1).reshape(-1)
    cc = torch.arange(cin).view(-1, 1, 1)
    oo = torch.arange(cout).view(1, -1, 1)
    tt = torch.arange(9).view(1, 1, -1)
    grad = (tt * gO * cin + oo * cin + cc).reshape(-1)
    return fwd.int(), dg.int(), grad.int()


def critic_maps(k1: int, C: int, npix: int):
    """Linear(C*npix -> k1) weight [k1, C*npix] (NCHW flatten f = c*npix + P): fwd B
    [npix][k1][C], dgrad B [npix][C][k1], gradient map param (k, f) -> dW [npix][k1][C]."""
    P = torch.arange(npix).view(-1, 1, 1)
    k = torch.arange(k1).view(1, -1, 1)
    c = torch.arange(C).view(1, 1, -1)
    fwd = (k * C * npix + c * npix + P).reshape(-1)
    c2 = torch.arange(C).view(1, -1, 1)
    k2 = torch.arange(k1).view(1, 1, -1)
    dg = (k2 * C * npix + c2 * npix + P).reshape(-1)
    kk = torch.arange(k1).view(-1, 1, 1)
    cc = torch.arange(C).view(1, -1, 1)
    pp = torch.arange(npix).view(1, 1, -1)
    grad = (pp * k1 * C + kk * C + cc).reshape(-1)
    return fwd.int(), dg.int(), grad.int()


def _pgrad(p) -> torch.Tensor:
    from .optim import grad_out
    return grad_out(p)


# ============================================================================ plan
class _Layer:
    pass


class PixPlan:
    """Pair tables, weight-packing maps and gradient maps of every GridNet layer for a padded
    map ph x pw (built once per model and device)."""

    def __init__(self, convs, convts, lin1, lin2, ph: int, pw: int, crop, device):
        self.device = torch.device(device)
        self.convs, self.convts, self.lin1, self.lin2 = convs, convts, lin1, lin2
        dev = self.device
        self.enc = []
        H, W = ph, pw
        for i, c in enumerate(convs):
            L = _Layer()
            L.H, L.W = H, W
            L.cout, L.cin = c.weight.shape[0], c.weight.shape[1]
            fwd, dg, wg = conv_pairs(H, W)
            L.tf, L.td, L.tw = pconv_table(fwd, dev), pconv_table(dg, dev), wgrad_table(wg, dev)
            L.mean_pairs = sum(len(e) for _, e in fwd) / len(fwd)
            L.cin_p = _ceil32(L.cin)
            fm, dm, gm, L.cop = conv_maps(L.cout, L.cin)
            if L.cin_p != L.cin:      # first layer (bit planes): K per pair padded to 32
                t = torch.arange(9).view(9, 1, 1)
                o = torch.arange(L.cout).view(1, -1, 1)
                cc = torch.arange(L.cin_p).view(1, 1, -1)
                fm = torch.where(cc < L.cin, o * L.cin * 9 + cc * 9 + t, -1).reshape(-1).int()
                oo = torch.arange(L.cout).view(-1, 1, 1)
                c3 = torch.arange(L.cin).view(1, -1, 1)
                tt = torch.arange(9).view(1, 1, -1)
                gm = (tt * L.cout * L.cin_p + oo * L.cin_p + c3).reshape(-1).int()
            L.fmap, L.dmap, L.gmap = fm.to(dev), dm.to(dev), gm.to(dev)
            L.fshape, L.dshape = (9, L.cout, L.cin_p), (9, L.cin_p, L.cop)
            # input gradient as a forward conv over dY: tap (ky, kx) uses W[2-ky, 2-kx]^T
            L.dmap_flip = dm.view(9, -1, L.cop).flip(0).reshape(-1).contiguous().to(dev)
            self.enc.append(L)
            H, W = (H + 1) // 2, (W + 1) // 2
        self.zh, self.zw = H, W
        self.dec = []
        for j, t in enumerate(convts):
            L = _Layer()
            L.H, L.W = H, W
            L.cin, L.cout = t.weight.shape[0], t.weight.shape[1]
            last = j == len(convts) - 1
            L.crop = crop if last else None
            fwd, dg, wg = convt_pairs(H, W, L.crop)
            L.npix_out = len(fwd)
            L.tf, L.td, L.tw = pconv_table(fwd, dev), pconv_table(dg, dev), wgrad_table(wg, dev)
            L.mean_pairs = sum(len(e) for _, e in fwd) / len(fwd)
            L.gO = LOGIT_LD if last else L.cout       # channel count of the output gradient
            fm, dm, gm = convt_maps(L.cin, L.cout, L.gO)
            L.fmap, L.dmap, L.gmap = fm.to(dev), dm.to(dev), gm.to(dev)
            L.fshape, L.dshape = (9, L.cout, L.cin), (9, L.cin, L.gO)
            self.dec.append(L)
            H, W = 2 * H, 2 * W
        k1 = lin1.weight.shape[0]
        zc = convs[-1].weight.shape[0]
        npix = self.zh * self.zw
        assert lin1.weight.shape[1] == zc * npix
        L = _Layer()
        L.k1, L.C, L.npix = k1, zc, npix
        fwd, dg, wg = critic_pairs(npix)
        L.tf, L.td, L.tw = pconv_table(fwd, dev), pconv_table(dg, dev), wgrad_table(wg, dev)
        L.mean_pairs = 1.0      # one tap per z pixel per output row: the per-tap form
        fm, dm, gm = critic_maps(k1, zc, npix)
        L.fmap, L.dmap, L.gmap = fm.to(dev), dm.to(dev), gm.to(dev)
        L.fshape, L.dshape = (npix, k1, zc), (npix, zc, k1)
        self.crit = L
        self.w2map = torch.arange(lin2.weight.numel(), dtype=torch.int32, device=dev)
        # the bit-plane first layer on conv.hip's stage-0 kernels (pooled conv + argmax,
        # band-layout wgrad) when it is the 32-channel layer those kernels implement
        self.enc0 = None
        c0 = convs[0]
        if (self.device.type == "cuda" and c0.weight.shape[0] == 32
                and c0.weight.shape[1] <= 32):
            from .encoder import HipEncoder
            self.enc0 = HipEncoder(ph, pw, c0.weight.shape[1], channels=(32,), device=dev)

    def pack(self, with_dgrad: bool):
        """bf16 B operands of every layer (one map_gather launch)"""
        segs, out = [], {"enc": [], "dec": []}

        def seg(p, m, shape):
            t = torch.empty(shape, dtype=_BF, device=self.device)
            segs.append((p.detach(), t, m))
            return t

        for i, (c, L) in enumerate(zip(self.convs, self.enc)):
            fw = seg(c.weight, L.fmap, L.fshape) if not (i == 0 and self.enc0 is not None) \
                else None
            dw = None
            if with_dgrad and i > 0:
                dw = seg(c.weight, L.dmap_flip if _imgconv_ok(L, self.device) else L.dmap,
                         L.dshape)
            out["enc"].append((fw, dw))
        for t, L in zip(self.convts, self.dec):
            out["dec"].append((seg(t.weight, L.fmap, L.fshape),
                               seg(t.weight, L.dmap, L.dshape) if with_dgrad else None))
        L = self.crit
        out["w1"] = seg(self.lin1.weight, L.fmap, L.fshape)
        out["w1d"] = seg(self.lin1.weight, L.dmap, L.dshape) if with_dgrad else None
        out["w2"] = seg(self.lin2.weight, self.w2map, self.lin2.weight.shape)
        map_gather(segs)
        return out


# ============================================================================ network
def _bits_pbc(bits: torch.Tensor, h: int, w: int, ph: int, pw: int, C: int) -> torch.Tensor:
    """int32 bit-plane obs [n, h*w] -> PBC planes [ph*pw][n][C] (bits as channels, zero
    padding outside the map); the generic first layer's input"""
    n = bits.shape[0]
    sh = torch.arange(min(C, 32), device=bits.device, dtype=torch.int32)
    x = ((bits.view(n, h, w, 1) >> sh) & 1).to(_BF)
    out = torch.zeros(ph, pw, n, C, dtype=_BF, device=bits.device)
    out[:h, :w, :, :x.shape[-1]] = x.permute(1, 2, 0, 3)
    return out.view(ph * pw, n, C)


class _GridNetPBC(torch.autograd.Function):
    """The whole GridNet forward / backward on the PBC layout. Returns (logits [h*w][n_s][96]
    bf16 pixel-major, value [n] fp32); its backward writes every parameter gradient into the
    parameter's flat slot (direct-gradient parameters)."""

    @staticmethod
    def forward(ctx, bits, plan, hw, n_s, grad, cells, *params):
        ctx.set_materialize_grads(False)
        h, w, ph, pw = hw
        n = bits.shape[0]
        dev = bits.device
        pk = plan.pack(grad)
        saved = {"pk": pk}
        # ---- encoder
        acts = []       # per encoder layer: its input operand (tensor, ps, bs, C, relu-on-load)
        pools = []      # per encoder layer: (pooled, idx) (layer 0 on conv.hip: (p, pidx))
        if plan.enc0 is not None and bits.is_cuda:
            L0 = plan.enc0.layers[0]
            c0 = plan.convs[0]
            plan.enc0.pack_layer(0, c0.weight.detach().contiguous())
            bp = torch.empty(n, ph * pw, dtype=torch.int32, device=dev)
            _N().check(_N().kernels().mbk_bits_pad(bits.contiguous().data_ptr(), n, h, w, ph, pw,
                                                   bp.data_ptr(), _N().stream_ptr()), "bits_pad")
            Ho, Wo = (ph + 1) // 2, (pw + 1) // 2
            pidx = torch.empty(n, Ho, Wo, L0.cout, dtype=torch.uint8, device=dev)
            p = plan.enc0._fwd(L0, bp, c0.bias.detach(), pool_idx=pidx)   # NHWC, pre-relu
            saved["bits_pad"] = bp
            acts.append(None)
            pools.append((p, pidx))
            x = (p, L0.cout, Ho * Wo * L0.cout, L0.cout, True)
            start = 1
        else:
            start = 0
            L = plan.enc[0]
            x0 = _bits_pbc(bits, h, w, ph, pw, L.cin_p)
            x = (x0, n * L.cin_p, L.cin_p, L.cin_p, False)
        for i in range(start, len(plan.enc)):
            L, c = plan.enc[i], plan.convs[i]
            y = torch.empty(L.H * L.W, n, L.cout, dtype=_BF, device=dev)
            if _imgconv_ok(L, dev):
                imgconv(x[0], x[1], x[2], x[3], pk["enc"][i][0], L.cout, n, y, n * L.cout,
                        L.cout, L.H, bias=c.bias.detach(), relu=True, a_relu=x[4])
            else:
                pconv(x[0], x[1], x[2], x[3], pk["enc"][i][0], L.tf, L.cout, n, y, n * L.cout,
                      L.cout, bias=c.bias.detach(), relu=True, a_relu=x[4])
            pooled, idx = ppool_fwd(y, L.H, L.W, n, L.cout)
            del y
            acts.append(x)
            pools.append((pooled, idx))
            x = (pooled, n * L.cout, L.cout, L.cout, False)
        z = x[0]                                               # [zh*zw][n][256]
        # ---- critic
        Lc = plan.crit
        hcrit = torch.empty(n, Lc.k1, dtype=_BF, device=dev)
        pconv(z, n * Lc.C, Lc.C, Lc.C, pk["w1"], Lc.tf, Lc.k1, n, hcrit, 0, Lc.k1,
              bias=plan.lin1.bias.detach(), relu=True)
        v = gemm_nt(hcrit, pk["w2"], plan.lin2.bias.detach(), out_dtype=torch.float32).view(-1)
        # ---- decoder (first n_s images)
        dx = [(z, n * Lc.C, Lc.C, Lc.C)]
        for j, (L, t) in enumerate(zip(plan.dec, plan.convts)):
            last = j == len(plan.dec) - 1
            xin = dx[-1]
            if last and cells is not None:   # active cells only: compact rows
                y = torch.empty(cells.cap, LOGIT_LD, dtype=_BF, device=dev)
                pconv(xin[0], xin[1], xin[2], xin[3], pk["dec"][j][0], L.tf, L.cout, n_s, y,
                      0, LOGIT_LD, bias=t.bias.detach(), cells=cells)
            elif last:
                y = torch.empty(L.npix_out, n_s, LOGIT_LD, dtype=_BF, device=dev)
                pconv(xin[0], xin[1], xin[2], xin[3], pk["dec"][j][0], L.tf, L.cout, n_s, y,
                      n_s * LOGIT_LD, LOGIT_LD, bias=t.bias.detach())
            else:
                y = torch.empty(L.npix_out, n_s, L.cout, dtype=_BF, device=dev)
                pconv(xin[0], xin[1], xin[2], xin[3], pk["dec"][j][0], L.tf, L.cout, n_s, y,
                      n_s * L.cout, L.cout, bias=t.bias.detach(), relu=True)
                dx.append((y, n_s * L.cout, L.cout, L.cout))
        logits = y
        ctx.plan, ctx.hw, ctx.n_s, ctx.n = plan, hw, n_s, n
        ctx.acts, ctx.pools, ctx.dx, ctx.hcrit, ctx.saved = acts, pools, dx, hcrit, saved
        ctx.cells = cells
        ctx.params = params
        return logits, v

    @staticmethod
    def backward(ctx, g_logits, g_value):
        plan, n_s, n = ctx.plan, ctx.n_s, ctx.n
        params = ctx.params
        pk = ctx.saved["pk"]
        dev = ctx.hcrit.device
        nconv = len(plan.enc)
        grads = [None] * len(params)
        # params: conv w/b x nconv, convt w/b x ndec, lin1 w/b, lin2 w/b

        def pg(i):
            grads[i] = _pgrad(params[i])
            return grads[i]

        # ---- critic
        Lc = plan.crit
        ic = 2 * nconv + 2 * len(plan.dec)
        dz_c = None
        if g_value is not None:
            dh = value_bwd(g_value.float().contiguous(), ctx.hcrit, params[ic + 2].detach(),
                           pg(ic + 2), pg(ic + 3))
            colsum(dh, Lc.k1, pg(ic + 1))
            z = ctx.dx[0][0]
            _wgrad(dh, 0, Lc.k1, Lc.k1, z, n * Lc.C, Lc.C, Lc.C, Lc, Lc.npix, n, pg(ic))
            dz_c = torch.empty(Lc.npix, n, Lc.C, dtype=_BF, device=dev)
            pconv(dh, 0, Lc.k1, Lc.k1, pk["w1d"], Lc.td, Lc.C, n, dz_c, n * Lc.C, Lc.C)
        # ---- decoder
        dz_d = None
        if g_logits is not None:
            g = g_logits.contiguous()
            gC = LOGIT_LD
            cells = ctx.cells
            for j in range(len(plan.dec) - 1, -1, -1):
                L = plan.dec[j]
                iw = 2 * nconv + 2 * j
                xin = ctx.dx[j]
                cin = L.cin
                gx = torch.empty(L.H * L.W, n_s, cin, dtype=_BF, device=dev)
                # relu mask of the input (a decoder output); the pooled code z is masked by the
                # pool backward
                mask = xin[0] if j > 0 else None
                if j == len(plan.dec) - 1 and cells is not None:
                    # sparse logits layer: g = compact rows of the active cells
                    cells.rows_colsum(g, gC, L.cout, pg(iw + 1))
                    pwgrad(g, 0, gC, gC, xin[0], xin[1], xin[2], xin[3], L.tw, n_s, L.gmap,
                           pg(iw), cells=cells)
                    pconv(g, 0, gC, gC, pk["dec"][j][1], L.td, cin, n_s, gx, n_s * cin, cin,
                          mask=mask, gather=cells)
                else:
                    colsum(g.view(-1, gC), L.cout, pg(iw + 1))
                    _wgrad(g, n_s * gC, gC, gC, xin[0], xin[1], xin[2], xin[3], L, 9, n_s,
                           pg(iw))
                    pconv(g, n_s * gC, gC, gC, pk["dec"][j][1], L.td, cin, n_s, gx, n_s * cin,
                          cin, mask=mask)
                g, gC = gx, cin
            dz_d = g
        # ---- encoder
        g1, n1, g2, n2 = dz_d, n_s, dz_c, n
        if g1 is None:
            g1, n1, g2, n2 = g2, n2, None, 0
        for i in range(nconv - 1, -1, -1):
            L = plan.enc[i]
            iw = 2 * i
            pooled, idx = ctx.pools[i]
            if i == 0 and plan.enc0 is not None and ctx.acts[0] is None:
                # conv.hip first layer: g1 is its (relu-masked) NHWC pooled gradient
                L0 = plan.enc0.layers[0]
                pidx = idx
                dc = torch.empty(n, L0.H, L0.W, L0.cout, dtype=_BF, device=dev)
                k = _N().kernels()
                _N().check(k.mbk_pool_bwd_idx(pidx.data_ptr(), g1.data_ptr(), n, L0.H, L0.W,
                                              L0.cout, dc.data_ptr(), _N().stream_ptr()),
                           "pool_bwd_idx")
                plan.enc0._wgrad(L0, ctx.saved["bits_pad"], dc, pg(0), pg(1))
                break
            if g1 is None:
                break
            dy = ppool_bwd(g1, n1, g2, n2, pooled, idx, L.H, L.W, n, L.cout)
            xa = ctx.acts[i]
            if _imgconv_ok(L, dev):
                imgwgrad(dy, n * L.cout, L.cout, L.cout, xa[0], xa[1], xa[2], xa[3], n, L.gmap,
                         pg(iw), L.H, x_relu=xa[4], bias_out=pg(iw + 1))
            else:
                _wgrad(dy, n * L.cout, L.cout, L.cout, xa[0], xa[1], xa[2], xa[3], L, 9, n,
                       pg(iw), x_relu=xa[4], bias_out=pg(iw + 1))
            if i == 0:
                break
            if i == 1 and plan.enc0 is not None and ctx.acts[0] is None:
                # input gradient straight into the first layer's NHWC layout, relu-masked by
                # its pre-relu pooled output
                p = ctx.pools[0][0]
                gx = torch.empty_like(p)
                if _imgconv_ok(L, dev):
                    imgconv(dy, n * L.cout, L.cout, L.cout, pk["enc"][i][1], L.cin, n, gx,
                            xa[1], xa[2], L.H, mask=p)
                else:
                    pconv(dy, n * L.cout, L.cout, L.cout, pk["enc"][i][1], L.td, L.cin, n, gx,
                          xa[1], xa[2], mask=p)
            else:
                gx = torch.empty(L.H * L.W, n, L.cin, dtype=_BF, device=dev)
                if _imgconv_ok(L, dev):
                    imgconv(dy, n * L.cout, L.cout, L.cout, pk["enc"][i][1], L.cin, n, gx,
                            n * L.cin, L.cin, L.H)
                else:
                    pconv(dy, n * L.cout, L.cout, L.cout, pk["enc"][i][1], L.td, L.cin, n, gx,
                          n * L.cin, L.cin)
            g1, n1, g2, n2 = gx, n, None, 0
        return (None, None, None, None, None, None) + tuple(grads)


def gridnet_pbc(plan: PixPlan, bits: torch.Tensor, h: int, w: int, ph: int, pw: int,
                n_logits: int | None = None, cells: Cells | None = None):
    """(logits [h*w][n_s][96] bf16 pixel-major, value fp32 [n]) of int32 bit-plane obs
    [n, h*w]; the decoder runs on the first n_s = n_logits (default n) observations. With
    ``cells`` (the active cells of those n_s samples) the logits are the compact rows
    [cells.cap][96] of the active cells only."""
    if cells is not None:
        assert cells.n == (bits.shape[0] if n_logits is None else n_logits) and cells.S == h * w
    n = bits.shape[0]
    n_s = n if n_logits is None else n_logits
    params = []
    for c in plan.convs:
        params += [c.weight, c.bias]
    for t in plan.convts:
        params += [t.weight, t.bias]
    params += [plan.lin1.weight, plan.lin1.bias, plan.lin2.weight, plan.lin2.bias]
    grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
    return _GridNetPBC.apply(bits.reshape(n, h * w).contiguous(), plan, (h, w, ph, pw), n_s,
                             grad, cells, *params)


def pbc_to_cell_major(logits: torch.Tensor) -> torch.Tensor:
    """[S][n][>=78] pixel-major logits -> [n, S*78] cell-major (fp32)"""
    S, n = logits.shape[:2]
    return logits[:, :, :78].float().permute(1, 0, 2).reshape(n, S * 78)
