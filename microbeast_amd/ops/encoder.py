"""IMPALA-CNN conv trunk on the HIP MFMA conv kernels (``conv.hip``).

Reference trunk: 3 x ConvSequence(conv -> maxpool -> res -> res)
(model.py:77-107, 56-73, 119-123). On device this runs as 15 fused conv
launches forward (relu / bias / residual / pool / bit-plane input folded in)
and 12 dgrad + 15 wgrad launches backward, all NHWC bf16 with fp32
accumulation, plus ONE weight-pack launch per call that converts the fp32
master parameters into the kernels' packed bf16 layouts.

Saved for backward per stage: the stage input, the pooled argmax (one byte
per pooled output), the pooled output and each residual block's input and
inner conv output.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from .. import _native as N
from .optim import grad_out


@dataclass
class ConvLayer:
    cin: int        # kernel input channels (27 -> 32 for the bit-plane input)
    cin_real: int   # parameter input channels
    cout: int
    H: int          # input spatial size
    W: int
    bits: bool      # input is the uint32 observation bit planes
    relu_in: bool
    pool: bool      # stage conv followed by maxpool(3,2,1)
    w_off: int = 0  # offsets into the packed buffers (elements)
    wb_off: int = -1


class _Job(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("fwd", ctypes.c_void_p), ("bwd", ctypes.c_void_p),
                ("cin", ctypes.c_int), ("cin_real", ctypes.c_int), ("cout", ctypes.c_int)]


class _RJob(ctypes.Structure):  # conv.hip MbkReduceJob
    _fields_ = [("partial", ctypes.c_void_p), ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p),
                ("nparts", ctypes.c_int), ("cin", ctypes.c_int), ("cin_real", ctypes.c_int),
                ("cout", ctypes.c_int), ("accumulate", ctypes.c_int)]


class _Job8(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("q", ctypes.c_void_p), ("scale", ctypes.c_void_p),
                ("cin", ctypes.c_int), ("cin_real", ctypes.c_int), ("cout", ctypes.c_int)]


def _nch(c: int) -> int:
    return 5 if c == 16 else 9


_PF_FWD = 8 * 256    # conv_fwd register-prefetch capacity (elements per group)
_PF_WGRAD = 4 * 256  # conv_wgrad prefetch capacity, X and dY each
# conv_fwd workgroup sizing (tools/microbench.py sweeps): LDS budget per workgroup (48 KB =
# 3 workgroups per CU) and the target output pixels per image group
_FWD_LDS = 48 * 1024
_FWD_PIX = 512
# res_bwd32 round size: output pixels per round and the LDS budget (KB) of its four tiles
# (maps of <= 2x2 pixels are mostly halo: their own budget)
_RES32_PIX = 256
_RES32_LDS_KB = 100
_RES32_LDS_KB_SMALL = 150


def _imgs_fwd(layer: ConvLayer, cin: int, cout: int, bits: bool, pool: bool,
              fp8: bool = False) -> int:
    """Images per workgroup iteration: ~512 output pixels, <= 48 KB LDS (3 WGs / CU), and
    one group's interior fits the register prefetch."""
    hw = layer.H * layer.W
    epp = 1 if bits else cin // 8
    pixb = (cin + 8) if fp8 else (cin * 2 + 16)  # bit planes are expanded in LDS
    imgs = max(1, _FWD_PIX // hw)
    while imgs > 1:
        sm = imgs * (layer.H + 2) * (layer.W + 2) * pixb + (imgs * hw * (cout + 4) * 2 if pool else 0)
        if sm <= _FWD_LDS and imgs * hw * epp <= _PF_FWD:
            break
        imgs //= 2
    return imgs


def _imgs_wgrad(layer: ConvLayer, unpool: bool = False, unpool_imgs: int = 2) -> int:
    hw = layer.H * layer.W
    xepp = 1 if layer.bits else layer.cin // 8
    dch = layer.cout // 8
    imgs = max(1, min(_PF_WGRAD // (hw * xepp), _PF_WGRAD // (hw * dch)))
    # LDS per image: conv.hip wg_tile_bytes (band layout on 8 / 16 / 24-wide maps pads the rows)
    if layer.W in (8, 16, 24) and layer.H % 4 == 0:
        rbx = (layer.W + 2) * layer.cin * 2 + (32 if layer.cin == 32 else 64)
        rbd = layer.W * layer.cout * 2 + (32 if layer.cout == 32 else 128)
        # (cin > cout: the tap-shifted dY tile has a zero halo: H + 2 rows)
        per = (layer.H + 2) * rbx + (layer.H + (2 if layer.cin > layer.cout else 0)) * rbd
    else:
        per = (layer.H + 2) * (layer.W + 2) * layer.cin * 2 + hw * layer.cout * 2
    if unpool:  # the pool-fused form scatters 2 images per round (one per 32-lane half)
        imgs = min(imgs, unpool_imgs)
    # (the halo'd dY tile is ~4 % larger: the stage-0 form keeps its 2 images per round, two
    # workgroups per CU still fit)
    lim = (72 if layer.cin > layer.cout else 64) * 1024
    while imgs > 1:
        if imgs * per <= lim:
            break
        imgs //= 2
    return imgs


class HipEncoder:
    """Owns layer geometry, packed-weight buffers and backward workspace."""

    def __init__(self, h: int, w: int, planes: int, channels=(16, 32, 32), device=None,
                 fp8: bool = False):
        assert planes <= 32, "bit-plane observations carry at most 32 planes"
        self.layers: list[ConvLayer] = []
        H, W, cin, cin_real, bits = h, w, 32, planes, True
        for co in channels:
            self.layers.append(ConvLayer(cin, cin_real, co, H, W, bits, False, True))
            H, W = (H + 1) // 2, (W + 1) // 2
            for _ in range(4):
                self.layers.append(ConvLayer(co, co, co, H, W, False, True, False))
            cin, cin_real, bits = co, co, False
        self.out_hw = (H, W)
        self.out_c = channels[-1]
        off = boff = 0
        for i, L in enumerate(self.layers):
            L.w_off = off
            off += L.cout * _nch(L.cin) * 32
            if i > 0:  # the observation layer needs no input gradient
                L.wb_off = boff
                boff += L.cin * _nch(L.cout) * 32
        self.packed_fwd = torch.zeros(off, dtype=torch.bfloat16, device=device)
        # acting forward: layers 1..14 in one fused launch (trunk.hip) when the trunk is the
        # reference (16, 32, 32) shape
        self.fused_tail = (tuple(channels) == (16, 32, 32) and self.layers[1].H <= 16
                           and self.layers[1].W <= 16)
        # Fused residual kernels (resblock.hip). Each flag selects the fused launch over the
        # per-layer conv_fwd / conv_wgrad composition it is bit-identical to (forward) or
        # checked against (backward); the per-layer path is what the parity tests compare
        # with (tests/test_gpu_conv.py), not a tuning knob.
        # 16-channel residual blocks (stage 0): one fused backward launch per block instead
        # of wgrad1 / dgrad1 / wgrad0 / dgrad0
        self.fused_res_bwd = True
        # 32-channel residual blocks (stages 1-2): one fused backward launch per block
        self.fused_res_bwd32 = True
        self.fused_res_fwd = True
        self.fused_res_fwd32 = True
        # the stage-0 residual kernel also runs stage 1's conv + pool
        self.fused_stage_fwd = True
        # the 32 -> 32 stage conv + pool on 4x4 maps: wave-owned images, no workgroup barriers
        self.fused_pool_fwd4 = True
        # 32-channel residual blocks on 4x4 / 2x2 maps with wave-owned 16-pixel blocks
        self.fused_res_blk32_wave = True
        # their backward on 4x4 / 2x2 maps by wave teams (stager + dW1, du, dx, dW0) synchronised
        # by LDS flags instead of workgroup rounds
        self.fused_res_bwd32_team = True
        # the observation layer's weight gradient expands the max-pool backward in its own
        # LDS staging (16-wide maps; bit-identical): no pool_bwd_idx launch, no 4.3 GB
        # full-resolution gradient in HBM per 524K-frame update
        self.fused_pool_wgrad0 = True
        # images per round of the pool-fused stage-0 weight gradient: 1 (36 KB of LDS, so two
        # of its workgroups fit beside an acting one under the backward cap: learner 17.63 ->
        # 16.94 ms at cap 1, bwd inside the bench 16.3 -> 15.4 ms over 3 seed pairs, profile
        # 45); 2 fills both 32-lane halves of its scatter but needs 70 KB
        self.wgrad0_imgs = 1
        # the 16 -> 32 stage conv on 8x8 maps: pool backward, weight gradient and input
        # gradient in one launch (stagebwd.hip; no full-resolution gradient in HBM)
        self.fused_pool_conv_bwd = True
        # one batched weight-gradient reduce per backward pass instead of one per layer
        self.defer_reduce = True
        # partial-row buffers of the weight gradients, one per layer (a backward pass defers
        # every reduce to one batched launch at its end: mbk_wgrad_reduce_batch)
        self._pbufs = {}
        self._rjobs = None  # list while a backward pass defers its reduces
        self.packed_bwd = torch.zeros(max(boff, 1), dtype=torch.bfloat16, device=device)
        # fp8 inference path (BASELINE config 5): e4m3 weights + per-channel scales
        self.fp8 = fp8
        # fp8 layers 1..14 in one fused launch (False: the 14 per-layer fp8 launches)
        self.fused_tail8 = True
        self.packed_fwd8 = torch.zeros(off, dtype=torch.uint8, device=device)
        self.scale8 = torch.zeros(sum(L.cout for L in self.layers), dtype=torch.float32,
                                  device=device)
        self._s_off = []
        so = 0
        for L in self.layers:
            self._s_off.append(so)
            so += L.cout

    # ------------------------------------------------------------ helpers
    def pack(self, weights: list[torch.Tensor], with_bwd: bool) -> None:
        k = N.kernels()
        for c0 in range(0, len(self.layers), 16):  # one launch packs up to 16 layers
            layers = self.layers[c0:c0 + 16]
            jobs = (_Job * len(layers))()
            for i, (L, wt) in enumerate(zip(layers, weights[c0:c0 + 16])):
                assert wt.dtype == torch.float32 and wt.is_contiguous()
                bwd = ((self.packed_bwd.data_ptr() + 2 * L.wb_off)
                       if (with_bwd and L.wb_off >= 0) else None)
                jobs[i] = _Job(wt.data_ptr(), self.packed_fwd.data_ptr() + 2 * L.w_off, bwd,
                               L.cin, L.cin_real, L.cout)
            N.check(k.mbk_conv_pack(ctypes.cast(jobs, ctypes.c_void_p), len(layers),
                                    N.stream_ptr()), "conv_pack")

    def pack_layer(self, i: int, weight: torch.Tensor, with_bwd: bool = False) -> None:
        """Pack layer i's fp32 weight only (GridNet's first layer uses this encoder's stage-0
        conv alone, ops/pixconv.py)."""
        L = self.layers[i]
        assert weight.dtype == torch.float32 and weight.is_contiguous()
        bwd = ((self.packed_bwd.data_ptr() + 2 * L.wb_off)
               if (with_bwd and L.wb_off >= 0) else None)
        jobs = (_Job * 1)(_Job(weight.data_ptr(), self.packed_fwd.data_ptr() + 2 * L.w_off, bwd,
                               L.cin, L.cin_real, L.cout))
        N.check(N.kernels().mbk_conv_pack(ctypes.cast(jobs, ctypes.c_void_p), 1, N.stream_ptr()),
                "conv_pack")

    def pack_fp8(self, weights: list[torch.Tensor]) -> None:
        k = N.kernels()
        for c0 in range(0, len(self.layers), 16):
            idx = list(range(c0, min(c0 + 16, len(self.layers))))
            jobs = (_Job8 * len(idx))()
            for j, i in enumerate(idx):
                L, wt = self.layers[i], weights[i]
                assert wt.dtype == torch.float32 and wt.is_contiguous()
                jobs[j] = _Job8(wt.data_ptr(), self.packed_fwd8.data_ptr() + L.w_off,
                                self.scale8.data_ptr() + 4 * self._s_off[i], L.cin, L.cin_real,
                                L.cout)
            N.check(k.mbk_conv_pack_fp8(ctypes.cast(jobs, ctypes.c_void_p), len(idx),
                                        N.stream_ptr()), "conv_pack_fp8")

    def _fwd8(self, i: int, x, bias, add=None):
        """Inference conv i on the fp8 MFMA kernel (bf16 activations in / out)."""
        L = self.layers[i]
        n = x.shape[0]
        Ho, Wo = ((L.H + 1) // 2, (L.W + 1) // 2) if L.pool else (L.H, L.W)
        y = torch.empty(n, Ho, Wo, L.cout, dtype=torch.bfloat16, device=x.device)
        imgs = _imgs_fwd(L, L.cin, L.cout, L.bits, L.pool, fp8=True)
        N.check(N.kernels().mbk_conv_fwd_fp8(
            x.data_ptr(), int(L.bits), L.cin, L.cout, self.packed_fwd8.data_ptr() + L.w_off,
            self.scale8.data_ptr() + 4 * self._s_off[i], N.ptr(bias), N.ptr(add), y.data_ptr(),
            n, L.H, L.W, imgs, int(L.relu_in), int(L.pool), N.stream_ptr()), "conv_fwd_fp8")
        return y

    def _tail(self, p: torch.Tensor, bs: list[torch.Tensor], head=None, value_out=None):
        """Layers 1..14 on the fused trunk kernel (inference): p = stage-0 pooled output.
        head = (w5 NHWC bf16, b5, wc, bc): also network.5 + critic in the same launch;
        returns (f [n, 256] bf16, value [n] fp32) instead of the trunk output."""
        L1, Ll = self.layers[1], self.layers[-1]
        n = p.shape[0]
        base = self.packed_fwd.data_ptr()
        wp = (ctypes.c_void_p * 14)(*[base + 2 * L.w_off for L in self.layers[1:15]])
        bp = (ctypes.c_void_p * 14)(*[b.data_ptr() for b in bs[1:15]])
        k = N.kernels()
        if head is not None:
            w5, b5, wc, bc = head
            f = torch.empty(n, w5.shape[0], dtype=torch.bfloat16, device=p.device)
            v = (value_out if value_out is not None
                 else torch.empty(n, dtype=torch.float32, device=p.device))
            N.check(k.mbk_trunk_tail_fc(p.data_ptr(), ctypes.cast(wp, ctypes.c_void_p),
                                        ctypes.cast(bp, ctypes.c_void_p), n, L1.H, L1.W, None,
                                        w5.data_ptr(), b5.data_ptr(), wc.data_ptr(),
                                        bc.data_ptr(), w5.shape[0], f.data_ptr(), v.data_ptr(),
                                        N.stream_ptr()), "trunk_tail_fc")
            return f, v
        y = torch.empty(n, Ll.H, Ll.W, Ll.cout, dtype=torch.bfloat16, device=p.device)
        N.check(k.mbk_trunk_tail(p.data_ptr(), ctypes.cast(wp, ctypes.c_void_p),
                                 ctypes.cast(bp, ctypes.c_void_p), n, L1.H, L1.W,
                                 y.data_ptr(), N.stream_ptr()), "trunk_tail")
        return y

    def _tail8(self, p: torch.Tensor, bs: list[torch.Tensor]) -> torch.Tensor:
        """Layers 1..14 on the fused fp8 trunk kernel (trunk.hip trunk_tail8_kernel): the
        per-layer fp8 numerics of ``_fwd8`` in one launch; p = stage-0 pooled output (bf16)."""
        L1, Ll = self.layers[1], self.layers[-1]
        n = p.shape[0]
        base, sbase = self.packed_fwd8.data_ptr(), self.scale8.data_ptr()
        wp = (ctypes.c_void_p * 14)(*[base + L.w_off for L in self.layers[1:15]])
        sp = (ctypes.c_void_p * 14)(*[sbase + 4 * self._s_off[i] for i in range(1, 15)])
        bp = (ctypes.c_void_p * 14)(*[b.data_ptr() for b in bs[1:15]])
        y = torch.empty(n, Ll.H, Ll.W, Ll.cout, dtype=torch.bfloat16, device=p.device)
        N.check(N.kernels().mbk_trunk_tail_fp8(
            p.data_ptr(), ctypes.cast(wp, ctypes.c_void_p), ctypes.cast(sp, ctypes.c_void_p),
            ctypes.cast(bp, ctypes.c_void_p), n, L1.H, L1.W, y.data_ptr(), N.stream_ptr()),
            "trunk_tail_fp8")
        return y

    def _fwd(self, L: ConvLayer, x, bias, add=None, mask_src=None, y_full=None, dgrad=False,
             pool_idx=None):
        n = x.shape[0]
        if dgrad:
            # data gradient = conv with flipped/transposed weights at the layer's input size
            cin, cout, w = L.cout, L.cin, self.packed_bwd.data_ptr() + 2 * L.wb_off
            H, W = L.H, L.W
            bits, relu, pool = False, False, False
        else:
            cin, cout, w = L.cin, L.cout, self.packed_fwd.data_ptr() + 2 * L.w_off
            H, W, bits, relu, pool = L.H, L.W, L.bits, L.relu_in, L.pool
        Ho, Wo = ((H + 1) // 2, (W + 1) // 2) if pool else (H, W)
        y = torch.empty(n, Ho, Wo, cout, dtype=torch.bfloat16, device=x.device)
        imgs = _imgs_fwd(L, cin, cout, bits, pool)
        N.check(N.kernels().mbk_conv_fwd(
            x.data_ptr(), int(bits), cin, cout, w, N.ptr(bias), N.ptr(add), N.ptr(mask_src),
            y.data_ptr(), N.ptr(y_full), N.ptr(pool_idx), n, H, W, imgs, int(relu), int(pool),
            N.stream_ptr()), "conv_fwd")
        return y

    def _wgrad(self, L: ConvLayer, x, dy, dw: torch.Tensor, db: torch.Tensor, dp=None,
               pidx=None):
        """dy=None: dY is max_pool2d's backward of dp through the argmax bytes pidx, expanded
        in the kernel's staging (the stage-0 layer of a 16-wide map)."""
        n = x.shape[0]
        imgs = _imgs_wgrad(L, unpool=dy is None, unpool_imgs=self.wgrad0_imgs)
        # persistent grid: as many workgroups as the device keeps resident (<= rounds)
        nparts = N.kernels().mbk_conv_wgrad_parts(int(L.bits), L.cin, L.cout, n, L.H, L.W, imgs,
                                                  int(dy is None))
        if nparts < 1:
            raise RuntimeError(f"conv_wgrad: unsupported shape {L}")
        row = L.cout * 9 * L.cin + L.cout
        need = (nparts + (nparts + 31) // 32) * row  # + the two-level reduce's scratch rows
        part = self._partials(L, need, x.device)
        k = N.kernels()
        st = N.stream_ptr()
        N.check(k.mbk_conv_wgrad(x.data_ptr(), int(L.bits), L.cin, L.cout, N.ptr(dy),
                                 N.ptr(dp), N.ptr(pidx), part.data_ptr(), nparts, n,
                                 L.H, L.W, imgs, int(L.relu_in), st), "conv_wgrad")
        self._reduce(part.data_ptr(), nparts, L, dw, db)

    def _partials(self, L: ConvLayer, need: int, device) -> torch.Tensor:
        """Layer L's partial-row buffer (one shared buffer when reduces are not deferred)."""
        key = id(L) if self._rjobs is not None else None
        b = self._pbufs.get(key)
        if b is None or b.numel() < need or b.device != device:
            b = torch.empty(max(need, 1 << 20), dtype=torch.float32, device=device)
            self._pbufs[key] = b
        return b

    def _reduce(self, partial: int, nparts: int, L: ConvLayer, dw, db) -> None:
        """Sum nparts partial rows at ``partial`` into L's fp32 dw / db: now, or queued for the
        backward pass's one batched launch (bit-identical either way, conv.hip)."""
        job = _RJob(partial, dw.data_ptr(), db.data_ptr(), nparts, L.cin, L.cin_real, L.cout, 0)
        if self._rjobs is not None:
            self._rjobs.append(job)
            return
        N.check(N.kernels().mbk_wgrad_reduce_batch(ctypes.byref(job), 1, N.stream_ptr()),
                "wgrad_reduce_batch")

    def _flush_reduces(self) -> None:
        jobs, self._rjobs = self._rjobs, None
        if jobs:
            arr = (_RJob * len(jobs))(*jobs)
            N.check(N.kernels().mbk_wgrad_reduce_batch(ctypes.cast(arr, ctypes.c_void_p),
                                                      len(jobs), N.stream_ptr()),
                    "wgrad_reduce_batch")

    def _res_fwd16(self, li: int, p: torch.Tensor, bs: list[torch.Tensor], stage=None):
        """Both residual blocks of a 16-channel stage in one launch (resblock.hip): returns
        (u0, y0, u1, y1), bit-identical to four conv_fwd launches. stage (not None): the same
        launch also runs the next stage's conv + pool on y1 from LDS and returns
        (u0, y0, u1, y1, (p_next, pidx_next)); stage=True also writes the argmax bytes."""
        n, H, W, C = p.shape
        outs = [torch.empty_like(p) for _ in range(4)]
        base = self.packed_fwd.data_ptr()
        wp = (ctypes.c_void_p * 4)(*[base + 2 * self.layers[li + 1 + j].w_off for j in range(4)])
        bp = (ctypes.c_void_p * 4)(*[bs[li + 1 + j].data_ptr() for j in range(4)])
        k = N.kernels()
        if stage is None:
            N.check(k.mbk_res_fwd16(p.data_ptr(), *[o.data_ptr() for o in outs],
                                    ctypes.cast(wp, ctypes.c_void_p),
                                    ctypes.cast(bp, ctypes.c_void_p), n, H, W, 4,
                                    N.stream_ptr()), "res_fwd16")
            return outs
        Ln = self.layers[li + 5]
        Ho, Wo = (H + 1) // 2, (W + 1) // 2
        pn = torch.empty(n, Ho, Wo, Ln.cout, dtype=torch.bfloat16, device=p.device)
        pidx = (torch.empty(n, Ho, Wo, Ln.cout, dtype=torch.uint8, device=p.device)
                if stage else None)
        N.check(k.mbk_res_fwd16_stage(p.data_ptr(), *[o.data_ptr() for o in outs],
                                      ctypes.cast(wp, ctypes.c_void_p),
                                      ctypes.cast(bp, ctypes.c_void_p),
                                      base + 2 * Ln.w_off, bs[li + 5].data_ptr(),
                                      pn.data_ptr(), N.ptr(pidx), n, H, W, 4,
                                      N.stream_ptr()), "res_fwd16_stage")
        return (*outs, (pn, pidx))

    def _pool_conv_fwd4(self, L: ConvLayer, x, bias, pidx):
        """Pooled stage conv 32 -> 32 on 4x4 maps with wave-owned images (stage2.hip):
        bit-identical to the pooled conv_fwd launch."""
        n = x.shape[0]
        y = torch.empty(n, 2, 2, L.cout, dtype=torch.bfloat16, device=x.device)
        N.check(N.kernels().mbk_pool_conv_fwd4(x.data_ptr(), self.packed_fwd.data_ptr() + 2 * L.w_off,
                                               bias.data_ptr(), y.data_ptr(), N.ptr(pidx), n,
                                               N.stream_ptr()), "pool_conv_fwd4")
        return y

    def _res_blk32(self, l0: int, x: torch.Tensor, bs: list[torch.Tensor]):
        """One 32-channel residual block (layers l0, l0+1) in one launch (resblock.hip):
        returns (u, y), bit-identical to two conv_fwd launches."""
        n, H, W, C = x.shape
        u, y = torch.empty_like(x), torch.empty_like(x)
        base = self.packed_fwd.data_ptr()
        wp = (ctypes.c_void_p * 2)(*[base + 2 * self.layers[l0 + j].w_off for j in range(2)])
        bp = (ctypes.c_void_p * 2)(*[bs[l0 + j].detach().data_ptr() for j in range(2)])
        if self.fused_res_blk32_wave and H == W and W in (2, 4):
            N.check(N.kernels().mbk_res_blk32_fwd_wave(x.data_ptr(), u.data_ptr(), y.data_ptr(),
                                                       ctypes.cast(wp, ctypes.c_void_p),
                                                       ctypes.cast(bp, ctypes.c_void_p), n, H, W,
                                                       N.stream_ptr()), "res_blk32_fwd_wave")
            return u, y
        imgs = max(1, min(16, (80 * 1024) // (2 * (H + 2) * (W + 2) * 80)))
        N.check(N.kernels().mbk_res_blk32_fwd(x.data_ptr(), u.data_ptr(), y.data_ptr(),
                                              ctypes.cast(wp, ctypes.c_void_p),
                                              ctypes.cast(bp, ctypes.c_void_p), n, H, W, imgs,
                                              N.stream_ptr()), "res_blk32_fwd")
        return u, y

    def _res_bwd16(self, L0: ConvLayer, L1: ConvLayer, x, u, g, dw1, db1, dw0, db0):
        """Fused backward of a 16-channel residual block y = x + conv1(relu(conv0(relu x))),
        u = conv0(relu x): returns dx; writes both layers' weight / bias gradients."""
        n = x.shape[0]
        H, W = L0.H, L0.W
        k = N.kernels()
        imgs = max(1, min(8, (80 * 1024) // (4 * (H + 2) * (W + 2) * 48)))
        dx = torch.empty_like(x)
        base = self.packed_bwd.data_ptr()
        nparts = k.mbk_res_bwd16_parts(n, H, W, imgs)
        if nparts < 1:
            raise RuntimeError(f"res_bwd16: unsupported shape {H}x{W}")
        need = k.mbk_res_bwd16_partial_floats(nparts)
        part = self._partials(L0, need, x.device)
        N.check(k.mbk_res_bwd16(x.data_ptr(), u.data_ptr(), g.data_ptr(), dx.data_ptr(),
                                base + 2 * L1.wb_off, base + 2 * L0.wb_off, part.data_ptr(),
                                nparts, None, None, None, None, n, H, W, imgs, 0,
                                N.stream_ptr()), "res_bwd16")
        self._reduce(part.data_ptr(), nparts, L1, dw1, db1)
        self._reduce(part.data_ptr() + 4 * (need // 2), nparts, L0, dw0, db0)
        return dx

    def _pool_conv_bwd(self, L: ConvLayer, dp, pidx, x, dw, db):
        """Backward of a pooled stage conv in one launch (stagebwd.hip): returns dx; writes the
        layer's weight / bias gradients."""
        n = x.shape[0]
        k = N.kernels()
        nparts = k.mbk_pool_conv_bwd_parts(n, L.cin, L.cout, L.H, L.W)
        need = k.mbk_pool_conv_bwd_partial_floats(nparts, L.cin, L.cout)
        part = self._partials(L, need, x.device)
        dx = torch.empty_like(x)
        N.check(k.mbk_pool_conv_bwd(dp.data_ptr(), pidx.data_ptr(), x.data_ptr(),
                                    self.packed_bwd.data_ptr() + 2 * L.wb_off, dx.data_ptr(),
                                    part.data_ptr(), nparts, None, None, n, L.cin, L.cout, L.H,
                                    L.W, 0, N.stream_ptr()), "pool_conv_bwd")
        self._reduce(part.data_ptr(), nparts, L, dw, db)
        return dx

    def _res_bwd32(self, L0: ConvLayer, L1: ConvLayer, x, u, g, dw1, db1, dw0, db0):
        """Fused backward of a 32-channel residual block (resblock.hip res_bwd32): returns dx;
        writes both layers' weight / bias gradients."""
        n = x.shape[0]
        H, W = L0.H, L0.W
        k = N.kernels()
        if self.fused_res_bwd32_team and H == W and W in (2, 4):
            # wave teams on 32-pixel items, no workgroup barriers (resblock.hip)
            dx = torch.empty_like(x)
            base = self.packed_bwd.data_ptr()
            nparts = k.mbk_res_bwd32_team_parts(n, H, W)
            need = k.mbk_res_bwd32_partial_floats(nparts)
            part = self._partials(L0, need, x.device)
            N.check(k.mbk_res_bwd32_team(x.data_ptr(), u.data_ptr(), g.data_ptr(), dx.data_ptr(),
                                         base + 2 * L1.wb_off, base + 2 * L0.wb_off,
                                         part.data_ptr(), nparts, n, H, W, N.stream_ptr()),
                    "res_bwd32_team")
            self._reduce(part.data_ptr(), nparts, L1, dw1, db1)
            self._reduce(part.data_ptr() + 4 * (need // 2), nparts, L0, dw0, db0)
            return dx
        lds_kb = _RES32_LDS_KB if H * W > 4 else _RES32_LDS_KB_SMALL
        imgs = max(1, min(_RES32_PIX // (H * W), (lds_kb * 1024 - 128) // (4 * (H + 2) * (W + 2) * 80)))
        dx = torch.empty_like(x)
        base = self.packed_bwd.data_ptr()
        nparts = k.mbk_res_bwd32_parts(n, H, W, imgs)
        if nparts < 1:
            raise RuntimeError(f"res_bwd32: unsupported shape {H}x{W}")
        need = k.mbk_res_bwd32_partial_floats(nparts)
        part = self._partials(L0, need, x.device)
        N.check(k.mbk_res_bwd32(x.data_ptr(), u.data_ptr(), g.data_ptr(), dx.data_ptr(),
                                base + 2 * L1.wb_off, base + 2 * L0.wb_off, part.data_ptr(),
                                nparts, None, None, None, None, n, H, W, imgs, 0,
                                N.stream_ptr()), "res_bwd32")
        self._reduce(part.data_ptr(), nparts, L1, dw1, db1)
        self._reduce(part.data_ptr() + 4 * (need // 2), nparts, L0, dw0, db0)
        return dx

    # ------------------------------------------------------------ passes
    def forward(self, obs_bits: torch.Tensor, params: list[torch.Tensor], save: bool,
                prepacked: bool = False, head=None, value_out=None):
        """params: [w0, b0, w1, b1, ...] fp32 in layer order. Returns (out NHWC bf16, saved).
        prepacked: the packed weight buffers are current (inference after pack_inference)."""
        ws, bs = params[0::2], params[1::2]
        x = obs_bits.contiguous()
        if self.fp8 and not save:
            if not prepacked:
                self.pack_fp8([w.detach() for w in ws])
            if self.fused_tail and self.fused_tail8:
                p = self._fwd8(0, x, bs[0].detach())
                return self._tail8(p, bs), []
            for st in range(len(self.layers) // 5):
                i = 5 * st
                p = self._fwd8(i, x, bs[i].detach())
                u0 = self._fwd8(i + 1, p, bs[i + 1].detach())
                y0 = self._fwd8(i + 2, u0, bs[i + 2].detach(), add=p)
                u1 = self._fwd8(i + 3, y0, bs[i + 3].detach())
                x = self._fwd8(i + 4, u1, bs[i + 4].detach(), add=y0)
            return x, []
        if not prepacked or save:
            self.pack([w.detach() for w in ws], with_bwd=save)
        if not save and self.fused_tail:
            p = self._fwd(self.layers[0], x, bs[0].detach())
            return self._tail(p, bs, head, value_out), []
        saved = []
        li = 0
        n = x.shape[0]
        nxt = None  # (p, pidx) of the next stage when the residual kernel ran its conv
        for _stage in range(len(self.layers) // 5):
            L = self.layers[li]
            Ho, Wo = (L.H + 1) // 2, (L.W + 1) // 2
            # pooled argmax (1 byte) instead of the full-resolution conv output
            pidx = (torch.empty(n, Ho, Wo, L.cout, dtype=torch.uint8, device=x.device)
                    if save else None)
            if nxt is not None:  # computed by the previous stage's fused residual kernel
                p, pidx = nxt
                nxt = None
            elif (self.fused_pool_fwd4 and x.is_cuda and L.cin == 32 and L.cout == 32
                  and L.pool and not L.bits and L.H == 4 and L.W == 4):
                p = self._pool_conv_fwd4(L, x, bs[li].detach(), pidx)
            else:
                p = self._fwd(L, x, bs[li].detach(), pool_idx=pidx)
            if self.fused_res_fwd and L.cout == 16 and p.is_cuda:
                Ln = self.layers[li + 5] if li + 5 < len(self.layers) else None
                if (self.fused_stage_fwd and Ln is not None and Ln.cin == 16 and Ln.cout == 32
                        and Ln.pool and not Ln.bits
                        # its pre-pool staging aliases the relu(u) tile (8x8, 5x5: fits;
                        # 12x12 with unpadded 64-byte staging rows)
                        and Ln.H * Ln.W * (64 if Ln.W == 12 else 72)
                        <= (Ln.H + 2) * (Ln.W + 2) * 48):
                    u0, y0, u1, y1, nxt = self._res_fwd16(li, p, [b.detach() for b in bs],
                                                          stage=save)
                else:
                    u0, y0, u1, y1 = self._res_fwd16(li, p, [b.detach() for b in bs])
            elif self.fused_res_fwd32 and L.cout == 32 and p.is_cuda:
                u0, y0 = self._res_blk32(li + 1, p, bs)
                u1, y1 = self._res_blk32(li + 3, y0, bs)
            else:
                u0 = self._fwd(self.layers[li + 1], p, bs[li + 1].detach())
                y0 = self._fwd(self.layers[li + 2], u0, bs[li + 2].detach(), add=p)
                u1 = self._fwd(self.layers[li + 3], y0, bs[li + 3].detach())
                y1 = self._fwd(self.layers[li + 4], u1, bs[li + 4].detach(), add=y0)
            if save:
                saved += [x, pidx, p, u0, y0, u1]
            x = y1
            li += 5
        return x, saved

    def backward(self, g: torch.Tensor, saved: list[torch.Tensor], params: list[torch.Tensor]):
        # each gradient goes straight into its parameter's flat slot when it can (optim.py)
        grads = [grad_out(p) for p in params]
        nst = len(self.layers) // 5
        g = g.contiguous()
        # the layers' partial-row reduces run as one batched launch at the end (30 small
        # launches off the backward's critical path; bit-identical sums)
        self._rjobs = [] if self.defer_reduce and g.is_cuda else None
        for s in range(nst - 1, -1, -1):
            li = 5 * s
            x, pidx, p, u0, y0, u1 = saved[6 * s:6 * s + 6]
            L = self.layers
            if self.fused_res_bwd and L[li + 1].cin == 16 and x.is_cuda:
                # both residual blocks of a 16-channel stage: one launch each (resblock.hip)
                dy0 = self._res_bwd16(L[li + 3], L[li + 4], y0, u1, g, grads[2 * (li + 4)],
                                      grads[2 * (li + 4) + 1], grads[2 * (li + 3)],
                                      grads[2 * (li + 3) + 1])
                dp = self._res_bwd16(L[li + 1], L[li + 2], p, u0, dy0, grads[2 * (li + 2)],
                                     grads[2 * (li + 2) + 1], grads[2 * (li + 1)],
                                     grads[2 * (li + 1) + 1])
            elif self.fused_res_bwd32 and L[li + 1].cin == 32 and x.is_cuda:
                dy0 = self._res_bwd32(L[li + 3], L[li + 4], y0, u1, g, grads[2 * (li + 4)],
                                      grads[2 * (li + 4) + 1], grads[2 * (li + 3)],
                                      grads[2 * (li + 3) + 1])
                dp = self._res_bwd32(L[li + 1], L[li + 2], p, u0, dy0, grads[2 * (li + 2)],
                                     grads[2 * (li + 2) + 1], grads[2 * (li + 1)],
                                     grads[2 * (li + 1) + 1])
            else:
                # res block 1: y1 = y0 + conv4(relu(u1)), u1 = conv3(relu(y0))
                self._wgrad(L[li + 4], u1, g, grads[2 * (li + 4)], grads[2 * (li + 4) + 1])
                du1 = self._fwd(L[li + 4], g, None, mask_src=u1, dgrad=True)
                self._wgrad(L[li + 3], y0, du1, grads[2 * (li + 3)], grads[2 * (li + 3) + 1])
                dy0 = self._fwd(L[li + 3], du1, None, mask_src=y0, add=g, dgrad=True)
                # res block 0
                self._wgrad(L[li + 2], u0, dy0, grads[2 * (li + 2)], grads[2 * (li + 2) + 1])
                du0 = self._fwd(L[li + 2], dy0, None, mask_src=u0, dgrad=True)
                self._wgrad(L[li + 1], p, du0, grads[2 * (li + 1)], grads[2 * (li + 1) + 1])
                dp = self._fwd(L[li + 1], du0, None, mask_src=p, add=dy0, dgrad=True)
            # maxpool + stage conv
            Ls = L[li]
            # the fused pool + weight-gradient kernel exists for the 16-wide stage-0 band
            # layout only: ask the library, else fall through to pool_bwd_idx
            if (s == 0 and Ls.bits and Ls.W == 16 and self.fused_pool_wgrad0 and x.is_cuda
                    and N.kernels().mbk_conv_wgrad_parts(
                        int(Ls.bits), Ls.cin, Ls.cout, x.shape[0], Ls.H, Ls.W,
                        _imgs_wgrad(Ls, True, self.wgrad0_imgs), 1) > 0):
                self._wgrad(Ls, x, None, grads[2 * li], grads[2 * li + 1], dp=dp, pidx=pidx)
                g = None
                continue
            if (s > 0 and self.fused_pool_conv_bwd and x.is_cuda
                    and N.kernels().mbk_pool_conv_bwd_parts(x.shape[0], Ls.cin, Ls.cout, Ls.H,
                                                            Ls.W) > 0):
                g = self._pool_conv_bwd(Ls, dp, pidx, x, grads[2 * li], grads[2 * li + 1])
                continue
            dc = torch.empty(pidx.shape[0], Ls.H, Ls.W, Ls.cout, dtype=torch.bfloat16,
                             device=pidx.device)
            N.check(N.kernels().mbk_pool_bwd_idx(pidx.data_ptr(), dp.data_ptr(), pidx.shape[0],
                                                 Ls.H, Ls.W, Ls.cout, dc.data_ptr(),
                                                 N.stream_ptr()), "pool_bwd_idx")
            self._wgrad(Ls, x, dc, grads[2 * li], grads[2 * li + 1])
            g = self._fwd(Ls, dc, None, dgrad=True) if s > 0 else None
        self._flush_reduces()
        return grads


class _EncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, obs_bits, enc: HipEncoder, *params):
        out, saved = enc.forward(obs_bits, list(params), save=True)
        ctx.enc = enc
        ctx.nsaved = len(saved)
        ctx.save_for_backward(*saved)
        ctx.params = params
        return out

    @staticmethod
    def backward(ctx, g):
        saved = list(ctx.saved_tensors)
        grads = ctx.enc.backward(g.to(torch.bfloat16), saved, list(ctx.params))
        return (None, None, *grads)


def encoder_params(network: torch.nn.Sequential, n_stages: int) -> list[torch.nn.Parameter]:
    """[w, b] per conv in HipEncoder layer order from a reference-named ``network``."""
    out = []
    for s in range(n_stages):
        cs = network[s]
        for conv in (cs.conv, cs.res_block0.conv0, cs.res_block0.conv1, cs.res_block1.conv0,
                     cs.res_block1.conv1):
            out += [conv.weight, conv.bias]
    return out


def encode(obs_bits: torch.Tensor, enc: HipEncoder, params: list[torch.Tensor],
           need_grad: bool, prepacked: bool = False, head=None, value_out=None):
    """NHWC bf16 trunk output [N, Ho, Wo, C] (head: (f, value) of the fused trunk head;
    value_out: the fp32 [N] buffer that value is written into)."""
    if need_grad:
        return _EncoderFn.apply(obs_bits, enc, *params)
    with torch.no_grad():
        return enc.forward(obs_bits, [p.detach() for p in params], save=False,
                           prepacked=prepacked, head=head, value_out=value_out)[0]
