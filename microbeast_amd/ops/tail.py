"""IMPALA trunk tail of the learner as ONE autograd node: relu -> network.5 -> relu ->
(sparse actor head score, critic), with every gradient written by our kernels.

Reference: model.py:119-137 (``network`` tail Linear + ReLU, ``actor``, ``critic``) and the
learner's scoring of the sampled actions (libs/utils.py:300-330).

Forward: ``mbk_fc_fwd`` (fc.hip) computes f = relu(W5 relu(y) + b5) (bf16) and the value
v = wc . f + bc in one pass over the trunk output y; the sparse head (ops/head.py) scores the
first ``n_score`` rows of f. Backward:

* the head's dX (fp32, first n_score rows) and the value gradient meet in ``mbk_value_bwd``
  (gridnet.hip): dh = (dv * wc + dX) * (f > 0), plus dWc / dbc -- no ATen add, no
  slice-backward zero fill, no dtype casts;
* dy = (dh . W5) * (y > 0): ``mbk_gemm_nt_mask`` (gemm.hip), the relu mask in the epilogue;
* dW5 = dh^T relu(y): ``mbk_fc_wgrad_ex`` with the relu applied while staging y;
* db5: ``mbk_colsum``; W5's NCHW<->NHWC column permutation both ways through index maps
  (``mbk_map_gather``), straight into the parameters' flat gradient slots.
"""
from __future__ import annotations


import torch

from .. import _native as N
from .pixconv import colsum, map_gather, value_bwd
from .optim import grad_out

_BF = torch.bfloat16
# head_dx_gather + value_bwd in one launch (False: the two separate launches, which the
# parity test compares against)
_FUSED_DX_VALUE = True


def nhwc_linear_maps(k1: int, c: int, hh: int, ww: int):
    """Linear(c*hh*ww -> k1) on an NHWC-flattened input, reference NCHW flatten of the weight
    [k1, c*hh*ww]: fwd B [k1, hh*ww*c] (NHWC columns), dgrad B [hh*ww*c, k1], grad map
    [k1*c*hh*ww] from the NHWC-ordered dW (int32 index maps)."""
    f = c * hh * ww
    k = torch.arange(k1).view(-1, 1, 1, 1)
    y = torch.arange(hh).view(1, -1, 1, 1)
    x = torch.arange(ww).view(1, 1, -1, 1)
    ch = torch.arange(c).view(1, 1, 1, -1)
    fwd = (k * f + ch * hh * ww + y * ww + x).reshape(k1, -1)         # [k1, hh, ww, c]
    dgrad = fwd.t().contiguous()
    kk = torch.arange(k1).view(-1, 1, 1, 1)
    cc = torch.arange(c).view(1, -1, 1, 1)
    yy = torch.arange(hh).view(1, 1, -1, 1)
    xx = torch.arange(ww).view(1, 1, 1, -1)
    grad = (kk * f + (yy * ww + xx) * c + cc).reshape(-1)            # dst (k, c, y, x)
    return fwd.int(), dgrad.int(), grad.int()


class TailMaps:
    """index maps of network.5's weight: NHWC-permuted fwd operand, its transpose (dgrad
    operand) and the NHWC dW -> parameter-layout map"""

    def __init__(self, out_features: int, c: int, ho: int, wo: int, device):
        fwd, dgrad, grad = nhwc_linear_maps(out_features, c, ho, wo)
        self.fwd, self.dgrad, self.grad = fwd.to(device), dgrad.to(device), grad.to(device)
        self.device = torch.device(device)
        self.key = (out_features, c, ho, wo)

    def pack(self, w5: torch.Tensor):
        wp = torch.empty(self.fwd.shape, dtype=_BF, device=w5.device)
        wt = torch.empty(self.dgrad.shape, dtype=_BF, device=w5.device)
        map_gather([(w5.detach(), wp, self.fwd), (w5.detach(), wt, self.dgrad)])
        return wp, wt


class _ImpalaTail(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, w5, b5, wc, bc, wa, ba, mask, action, n_score, head, maps, abits=None):
        ctx.set_materialize_grads(False)
        n = y.shape[0]
        y2 = y.reshape(n, -1)
        I = y2.shape[1]
        O = w5.shape[0]
        wp, wt = maps.pack(w5)
        f = torch.empty(n, O, dtype=_BF, device=y.device)
        v = torch.empty(n, dtype=torch.float32, device=y.device)
        N.check(N.kernels().mbk_fc_fwd(y2.data_ptr(), 1, wp.data_ptr(), b5.data_ptr(),
                                       wc.data_ptr(), bc.data_ptr(), n, I, O, f.data_ptr(),
                                       v.data_ptr(), N.stream_ptr()), "fc_fwd")
        fh = f[:n_score]
        head.pack(wa.detach(), ba.detach(), with_t=True)
        logp, ent = head.forward(fh, mask, action, sample=False, rng=None, abits=abits)
        ctx.save_for_backward(y2, f, wt, mask, action)
        ctx.meta = (head, maps, n_score, y.shape)
        ctx.params = (w5, b5, wc, bc, wa, ba)
        return logp, ent, v

    @staticmethod
    def backward(ctx, g_logp, g_ent, g_v):
        from .copy import zeros
        y2, f, wt, mask, action = ctx.saved_tensors
        head, maps, n_score, yshape = ctx.meta
        w5, b5, wc, bc, wa, ba = ctx.params
        n, I = y2.shape
        dev = y2.device
        if g_logp is None:
            g_logp = zeros(n_score, device=dev)
        if g_v is None:
            g_v = zeros(n, device=dev)
        gwa, gba = grad_out(wa), grad_out(ba)
        gwc, gbc = grad_out(wc), grad_out(bc)
        k = N.kernels()
        g_v = g_v.float().contiguous()
        if f.is_cuda and f.shape[1] == 256 and _FUSED_DX_VALUE:
            # head dX gather + critic backward in one pass (head.hip head_dx_value)
            partial = torch.empty(k.mbk_head_dx_value_parts(n), 257, dtype=torch.float32,
                                  device=dev)
            dh, _, _ = head.backward(f[:n_score], mask, action, g_logp.float().contiguous(),
                                     None if g_ent is None else g_ent.float().contiguous(),
                                     gwa, gba.view(-1), value=(g_v, f, wc.detach(), partial))
            colsum(partial, 257, gwc, 256, gbc)
        else:
            dX, _, _ = head.backward(f[:n_score], mask, action, g_logp.float().contiguous(),
                                     None if g_ent is None else g_ent.float().contiguous(),
                                     gwa, gba.view(-1))
            dh = value_bwd(g_v, f, wc.detach(), gwc, gbc, gadd=dX)
        st = N.stream_ptr()
        dy = torch.empty(n, I, dtype=_BF, device=dev)
        O = dh.shape[1]
        N.check(k.mbk_gemm_nt_mask(dh.data_ptr(), wt.data_ptr(), dy.data_ptr(), None, n, I, O, O,
                                   O, I, 0, 1, y2.data_ptr(), st), "gemm_nt_mask")
        dw5 = torch.empty(O, I, dtype=torch.float32, device=dev)
        gb5 = grad_out(b5)
        wparts = k.mbk_fc_wgrad_wide_parts(n, O, I)
        if wparts > 0:  # dW5 and db5 in one pass over dh / y2 (fc.hip fc_wgrad_wide_kernel)
            scratch = torch.empty((wparts + (wparts + 31) // 32) * (O * I + O),
                                  dtype=torch.float32, device=dev)
            N.check(k.mbk_fc_wgrad_wide(dh.data_ptr(), y2.data_ptr(), n, O, I, 1,
                                        scratch.data_ptr(), wparts, dw5.data_ptr(),
                                        gb5.data_ptr(), st), "fc_wgrad_wide")
        else:
            nparts = k.mbk_fc_wgrad_parts(n, O, I)
            scratch = torch.empty((nparts + (nparts + 31) // 32) * O * I, dtype=torch.float32,
                                  device=dev)
            N.check(k.mbk_fc_wgrad_ex(dh.data_ptr(), y2.data_ptr(), n, O, I, scratch.data_ptr(),
                                      nparts, dw5.data_ptr(), 0, 1, st), "fc_wgrad_ex")
            colsum(dh, O, gb5)
        gw5 = grad_out(w5)
        map_gather([(dw5, gw5, maps.grad)])
        return (dy.view(yshape), gw5, gb5, gwc, gbc, gwa, gba) + (None,) * 6


def impala_tail(y, fc, critic, actor, mask, action, n_score, head, maps, abits=None):
    """(logp [n_score], entropy [n_score], value [n]) of the trunk output y [n, ho, wo, c].
    abits: the scored frames' active-cell bitmap rows from the acting step (optional)."""
    return _ImpalaTail.apply(y, fc.weight, fc.bias, critic.weight, critic.bias, actor.weight,
                             actor.bias, mask, action, n_score, head, maps, abits)
