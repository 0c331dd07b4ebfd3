"""Masked multi-discrete microRTS action head (per-cell segmented softmax).

Reference: ``CategoricalMasked`` + the per-component loop of
``Agent.get_action`` (reference model.py:33-52, 165-216): logits of shape
(N, 78*s*s) are split by nvec=[6,4,4,4,4,7,49]*s*s, masked with
``where(mask, logits, -1e8)``, sampled / scored, and log-probs and entropies
are *summed* over all 7*s*s components per sample.

Device tensors go through the HIP kernels in ``csrc/kernels/masked_cell.hip``
(one thread per cell, LDS-staged); CPU tensors use a vectorised torch
formulation with identical semantics (it is also the test oracle). The fused
GEMM+epilogue variant lives in ``head.py``.
"""
from __future__ import annotations

import torch

from .. import _native as N

NVEC = (6, 4, 4, 4, 4, 7, 49)
OFFS = (0, 6, 10, 14, 18, 22, 29, 78)
CELL = 78
COMPS = 7
MASK_FILL = -1e8  # reference model.py:43


def unpack_mask(mask_bits: torch.Tensor) -> torch.Tensor:
    """int32 [..., 3] bit-packed mask -> bool [..., 78]."""
    m = mask_bits.to(torch.int64) & 0xFFFFFFFF
    j = torch.arange(CELL, device=mask_bits.device)
    word = m[..., (j // 32)]
    return ((word >> (j % 32)) & 1).bool()


def pack_mask(mask_bool: torch.Tensor) -> torch.Tensor:
    """bool [..., 78] -> int32 [..., 3] (inverse of unpack_mask)."""
    shape = mask_bool.shape[:-1]
    m = torch.zeros(*shape, 96, dtype=torch.int64, device=mask_bool.device)
    m[..., :CELL] = mask_bool.to(torch.int64)
    w = (m.view(*shape, 3, 32) << torch.arange(32, device=m.device)).sum(-1)
    w = torch.where(w >= 2**31, w - 2**32, w)
    return w.to(torch.int32)


# ---------------------------------------------------------------- torch formulation
def cell_head_torch(logits: torch.Tensor, mask: torch.Tensor, action: torch.Tensor | None,
                    generator: torch.Generator | None = None):
    """Vectorised reference semantics.

    logits: [N, S*78] float; mask: bool [N, S, 78] or int32 bits [N, S, 3];
    action: uint8/int64 [N, S, 7] to score, or None to sample.
    Returns (action [N,S,7] uint8, logp [N], entropy [N]) — differentiable in logits.
    """
    n = logits.shape[0]
    z = logits.float().view(n, -1, CELL)
    if mask.dtype != torch.bool:
        mask = unpack_mask(mask)
    mask = mask.view(n, -1, CELL)
    zm = torch.where(mask, z, torch.full_like(z, MASK_FILL))
    acts, lps, ents = [], [], []
    for k in range(COMPS):
        seg = zm[..., OFFS[k]:OFFS[k + 1]]
        mseg = mask[..., OFFS[k]:OFFS[k + 1]]
        logp_all = seg - torch.logsumexp(seg, dim=-1, keepdim=True)
        p = logp_all.exp()
        ents.append(-torch.where(mseg, p * logp_all, torch.zeros_like(p)).sum(-1))
        if action is None:
            with torch.no_grad():
                a = torch.multinomial(p.detach().reshape(-1, NVEC[k]), 1, generator=generator)
                a = a.view(n, -1)
        else:
            a = action[..., k].long()
        acts.append(a)
        lps.append(logp_all.gather(-1, a.unsqueeze(-1)).squeeze(-1))
    act = torch.stack(acts, -1).to(torch.uint8)
    logp = torch.stack(lps, -1).sum((1, 2))
    ent = torch.stack(ents, -1).sum((1, 2))
    return act, logp, ent


# ---------------------------------------------------------------- HIP kernels
def _cells(logits: torch.Tensor) -> tuple[int, int]:
    n = logits.shape[0]
    nc = logits.numel() // CELL
    return n, nc


def sample_gpu(logits: torch.Tensor, mask_bits: torch.Tensor, rng_state: torch.Tensor,
               action_out: torch.Tensor | None = None, cell_logp: torch.Tensor | None = None,
               logp_out: torch.Tensor | None = None):
    """Sample actions on device. rng_state: uint64-as-int64 [2] = (seed, step)."""
    k = N.kernels()
    logits = logits.contiguous()
    n, nc = _cells(logits)
    dev = logits.device
    if action_out is None:
        action_out = torch.empty(n, nc // n, COMPS, dtype=torch.uint8, device=dev)
    if cell_logp is None:
        cell_logp = torch.empty(nc, dtype=torch.float32, device=dev)
    if logp_out is None:
        logp_out = torch.empty(n, dtype=torch.float32, device=dev)
    st = N.stream_ptr()
    N.check(k.mbk_masked_cell_fwd(logits.data_ptr(), int(logits.dtype == torch.bfloat16),
                                  mask_bits.data_ptr(), action_out.data_ptr(), rng_state.data_ptr(),
                                  1, nc, cell_logp.data_ptr(), None, st), "masked_cell_fwd")
    N.check(k.mbk_row_sum(cell_logp.data_ptr(), n, nc // n, logp_out.data_ptr(), st), "row_sum")
    N.check(k.mbk_rng_advance(rng_state.data_ptr(), st), "rng_advance")
    return action_out, logp_out


class _ScoreGPU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, mask_bits, action):
        k = N.kernels()
        logits = logits.contiguous()
        n, nc = _cells(logits)
        dev = logits.device
        cl = torch.empty(nc, dtype=torch.float32, device=dev)
        ce = torch.empty(nc, dtype=torch.float32, device=dev)
        st = N.stream_ptr()
        N.check(k.mbk_masked_cell_fwd(logits.data_ptr(), int(logits.dtype == torch.bfloat16),
                                      mask_bits.data_ptr(), action.data_ptr(), None, 0, nc,
                                      cl.data_ptr(), ce.data_ptr(), st), "masked_cell_fwd")
        logp = torch.empty(n, dtype=torch.float32, device=dev)
        ent = torch.empty(n, dtype=torch.float32, device=dev)
        N.check(k.mbk_row_sum(cl.data_ptr(), n, nc // n, logp.data_ptr(), st), "row_sum")
        N.check(k.mbk_row_sum(ce.data_ptr(), n, nc // n, ent.data_ptr(), st), "row_sum")
        ctx.save_for_backward(logits, mask_bits, action)
        ctx.cps = nc // n
        return logp, ent

    @staticmethod
    def backward(ctx, g_logp, g_ent):
        logits, mask_bits, action = ctx.saved_tensors
        k = N.kernels()
        n, nc = _cells(logits)
        if g_logp is None:
            g_logp = torch.zeros(n, device=logits.device)
        if g_ent is None:
            g_ent = torch.zeros(n, device=logits.device)
        g_logp = g_logp.float().contiguous()
        g_ent = g_ent.float().contiguous()
        d = torch.empty_like(logits)
        N.check(k.mbk_masked_cell_bwd(logits.data_ptr(), int(logits.dtype == torch.bfloat16),
                                      mask_bits.data_ptr(), action.data_ptr(), g_logp.data_ptr(),
                                      g_ent.data_ptr(), ctx.cps, nc, d.data_ptr(),
                                      int(d.dtype == torch.bfloat16), N.stream_ptr()),
                "masked_cell_bwd")
        return d, None, None


# ---------------------------------------------------------------- pixel-major logits
# GridNet's decoder writes its logits pixel-major, [cell-of-map][sample][ld] bf16 (ld >= 78,
# ops/pixconv.py); these run the same masked-cell kernels with that row mapping, and the
# backward writes the logit gradient in the same layout (padding columns zero), which is the
# decoder backward's A operand as it is.
def _pbc_cm(logits: torch.Tensor) -> torch.Tensor:
    S, n = logits.shape[:2]
    return logits[:, :, :CELL].float().permute(1, 0, 2).reshape(n, S * CELL)


class _ScorePBC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, mask_bits, action):
        k = N.kernels()
        S, n, ld = logits.shape
        nc = S * n
        dev = logits.device
        assert logits.dtype == torch.bfloat16 and logits.is_contiguous()
        assert mask_bits.numel() == nc * 3 and action.numel() == nc * COMPS
        cl = torch.empty(nc, dtype=torch.float32, device=dev)
        ce = torch.empty(nc, dtype=torch.float32, device=dev)
        st = N.stream_ptr()
        N.check(k.mbk_masked_cell_fwd_pbc(logits.data_ptr(), S, n, ld, mask_bits.data_ptr(),
                                          action.data_ptr(), None, 0, nc, cl.data_ptr(),
                                          ce.data_ptr(), st), "masked_cell_fwd_pbc")
        logp = torch.empty(n, dtype=torch.float32, device=dev)
        ent = torch.empty(n, dtype=torch.float32, device=dev)
        N.check(k.mbk_row_sum(cl.data_ptr(), n, S, logp.data_ptr(), st), "row_sum")
        N.check(k.mbk_row_sum(ce.data_ptr(), n, S, ent.data_ptr(), st), "row_sum")
        ctx.save_for_backward(logits, mask_bits, action)
        return logp, ent

    @staticmethod
    def backward(ctx, g_logp, g_ent):
        logits, mask_bits, action = ctx.saved_tensors
        k = N.kernels()
        S, n, ld = logits.shape
        if g_logp is None:
            g_logp = torch.zeros(n, device=logits.device)
        if g_ent is None:
            g_ent = torch.zeros(n, device=logits.device)
        g_logp = g_logp.float().contiguous()
        g_ent = g_ent.float().contiguous()
        d = torch.empty_like(logits)
        N.check(k.mbk_masked_cell_bwd_pbc(logits.data_ptr(), S, n, ld, mask_bits.data_ptr(),
                                          action.data_ptr(), g_logp.data_ptr(), g_ent.data_ptr(),
                                          S * n, d.data_ptr(), N.stream_ptr()),
                "masked_cell_bwd_pbc")
        return d, None, None


def score_pbc(logits: torch.Tensor, mask_bits: torch.Tensor, action: torch.Tensor):
    """(logp [n], entropy [n]) of pixel-major logits [S][n][ld], differentiable in them."""
    if logits.is_cuda:
        return _ScorePBC.apply(logits, mask_bits.contiguous(), action.contiguous())
    _, lp, ent = cell_head_torch(_pbc_cm(logits), mask_bits, action)
    return lp, ent


def sample_pbc(logits: torch.Tensor, mask_bits: torch.Tensor, rng_state: torch.Tensor | None = None,
               generator: torch.Generator | None = None, action_out=None, cell_logp=None,
               logp_out=None):
    """(action [n,S,7] uint8, logp [n]) sampled from pixel-major logits [S][n][ld]."""
    S, n, ld = logits.shape
    if not logits.is_cuda:
        with torch.no_grad():
            a, lp, _ = cell_head_torch(_pbc_cm(logits), mask_bits, None, generator)
        return a, lp
    k = N.kernels()
    nc = S * n
    dev = logits.device
    assert logits.dtype == torch.bfloat16 and logits.is_contiguous()
    if action_out is None:
        action_out = torch.empty(n, S, COMPS, dtype=torch.uint8, device=dev)
    if cell_logp is None:
        cell_logp = torch.empty(nc, dtype=torch.float32, device=dev)
    if logp_out is None:
        logp_out = torch.empty(n, dtype=torch.float32, device=dev)
    assert action_out.numel() == nc * COMPS and cell_logp.numel() >= nc
    st = N.stream_ptr()
    N.check(k.mbk_masked_cell_fwd_pbc(logits.data_ptr(), S, n, ld, mask_bits.contiguous().data_ptr(),
                                      action_out.data_ptr(), rng_state.data_ptr(), 1, nc,
                                      cell_logp.data_ptr(), None, st), "masked_cell_fwd_pbc")
    N.check(k.mbk_row_sum_rng(cell_logp.data_ptr(), n, S, logp_out.data_ptr(),
                              rng_state.data_ptr(), st), "row_sum_rng")
    return action_out, logp_out


# ---------------------------------------------------------------- compact active-cell rows
# The sparse GridNet logits layer (ops/pixconv.py Cells) produces logits only for the active
# cells, as compact rows [cap][ld] bf16 (row r = cell cells.rowcell[r]); every other cell is
# fully masked (log-prob 0, entropy 0, gradient 0, sampled action 0).
def _rows_cm(Zc: torch.Tensor, cells) -> torch.Tensor:
    """compact rows -> cell-major [n, S*78] fp32 (zeros at inactive cells), differentiable"""
    nact = int(cells.totals[0])
    idx = cells.rowcell[:nact].long()
    cm = torch.zeros(cells.n * cells.S, CELL, dtype=torch.float32)
    cm = cm.index_copy(0, idx, Zc[:nact, :CELL].float())
    return cm.view(cells.n, cells.S * CELL)


def _zero(t: torch.Tensor):
    N.check(N.kernels().mbk_memset(t.data_ptr(), 0, t.numel() * t.element_size(), N.stream_ptr()),
            "memset")


class _ScoreRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Zc, cells, mask_bits, action):
        k = N.kernels()
        n, S = cells.n, cells.S
        nc = n * S
        dev = Zc.device
        ld = Zc.shape[-1]
        assert Zc.dtype == torch.bfloat16 and Zc.is_contiguous() and Zc.numel() == cells.cap * ld
        assert mask_bits.numel() == nc * 3 and action.numel() == nc * COMPS
        cl = torch.empty(nc, dtype=torch.float32, device=dev)
        ce = torch.empty(nc, dtype=torch.float32, device=dev)
        _zero(cl)
        _zero(ce)
        st = N.stream_ptr()
        nblk = max(1, min(8192, -(-cells.cap // 64)))
        N.check(k.mbk_masked_cell_rows_fwd(Zc.data_ptr(), ld, cells.rowcell.data_ptr(),
                                           cells.totals.data_ptr(), nblk, mask_bits.data_ptr(),
                                           action.data_ptr(), None, 0, cl.data_ptr(),
                                           ce.data_ptr(), st), "masked_cell_rows_fwd")
        logp = torch.empty(n, dtype=torch.float32, device=dev)
        ent = torch.empty(n, dtype=torch.float32, device=dev)
        N.check(k.mbk_row_sum(cl.data_ptr(), n, S, logp.data_ptr(), st), "row_sum")
        N.check(k.mbk_row_sum(ce.data_ptr(), n, S, ent.data_ptr(), st), "row_sum")
        ctx.save_for_backward(Zc, mask_bits, action)
        ctx.cells = cells
        return logp, ent

    @staticmethod
    def backward(ctx, g_logp, g_ent):
        Zc, mask_bits, action = ctx.saved_tensors
        cells = ctx.cells
        k = N.kernels()
        n = cells.n
        if g_logp is None:
            g_logp = torch.zeros(n, device=Zc.device)
        if g_ent is None:
            g_ent = torch.zeros(n, device=Zc.device)
        g_logp = g_logp.float().contiguous()
        g_ent = g_ent.float().contiguous()
        d = torch.empty_like(Zc)     # rows >= totals[0] are never read
        nblk = max(1, min(8192, -(-cells.cap // 64)))
        N.check(k.mbk_masked_cell_rows_bwd(Zc.data_ptr(), Zc.shape[-1], cells.rowcell.data_ptr(),
                                           cells.totals.data_ptr(), nblk, cells.S,
                                           mask_bits.data_ptr(), action.data_ptr(),
                                           g_logp.data_ptr(), g_ent.data_ptr(), d.data_ptr(),
                                           N.stream_ptr()), "masked_cell_rows_bwd")
        return d, None, None, None


def score_rows(Zc: torch.Tensor, cells, mask_bits: torch.Tensor, action: torch.Tensor):
    """(logp [n], entropy [n]) of compact active-cell logits, differentiable in them."""
    if Zc.is_cuda:
        return _ScoreRows.apply(Zc, cells, mask_bits.contiguous(), action.contiguous())
    _, lp, ent = cell_head_torch(_rows_cm(Zc, cells), mask_bits, action)
    return lp, ent


def sample_rows(Zc: torch.Tensor, cells, mask_bits: torch.Tensor,
                rng_state: torch.Tensor | None = None, generator: torch.Generator | None = None,
                action_out=None, cell_logp=None, logp_out=None):
    """(action [n,S,7] uint8, logp [n]) sampled from compact active-cell logits (same Philox
    draws as the dense kernel: keyed by cell index)."""
    n, S = cells.n, cells.S
    if not Zc.is_cuda:
        with torch.no_grad():
            a, lp, _ = cell_head_torch(_rows_cm(Zc, cells), mask_bits, None, generator)
        return a, lp
    k = N.kernels()
    nc = n * S
    dev = Zc.device
    if action_out is None:
        action_out = torch.empty(n, S, COMPS, dtype=torch.uint8, device=dev)
    if cell_logp is None:
        cell_logp = torch.empty(nc, dtype=torch.float32, device=dev)
    if logp_out is None:
        logp_out = torch.empty(n, dtype=torch.float32, device=dev)
    assert action_out.numel() == nc * COMPS and cell_logp.numel() >= nc
    _zero(action_out)
    _zero(cell_logp)
    st = N.stream_ptr()
    nblk = max(1, min(8192, -(-cells.cap // 64)))
    N.check(k.mbk_masked_cell_rows_fwd(Zc.data_ptr(), Zc.shape[-1], cells.rowcell.data_ptr(),
                                       cells.totals.data_ptr(), nblk,
                                       mask_bits.contiguous().data_ptr(), action_out.data_ptr(),
                                       rng_state.data_ptr(), 1, cell_logp.data_ptr(), None, st),
            "masked_cell_rows_fwd")
    N.check(k.mbk_row_sum_rng(cell_logp.data_ptr(), n, S, logp_out.data_ptr(),
                              rng_state.data_ptr(), st), "row_sum_rng")
    return action_out, logp_out


def score(logits: torch.Tensor, mask_bits: torch.Tensor, action: torch.Tensor):
    """(logp [N], entropy [N]) of given actions, differentiable in logits."""
    if logits.is_cuda:
        return _ScoreGPU.apply(logits, mask_bits.contiguous(), action.contiguous())
    _, lp, ent = cell_head_torch(logits, mask_bits, action)
    return lp, ent


def sample(logits: torch.Tensor, mask_bits: torch.Tensor, rng_state: torch.Tensor | None = None,
           generator: torch.Generator | None = None):
    """(action [N,S,7] uint8, logp [N]) sampled under the mask (no grad)."""
    if logits.is_cuda:
        return sample_gpu(logits, mask_bits.contiguous(), rng_state)
    with torch.no_grad():
        a, lp, _ = cell_head_torch(logits, mask_bits, None, generator)
    return a, lp


def greedy(logits: torch.Tensor, mask_bits: torch.Tensor) -> torch.Tensor:
    """Arg-max action per component under the mask (evaluation), uint8 [N,S,7]."""
    n = logits.shape[0]
    z = logits.float().view(n, -1, CELL)
    mask = unpack_mask(mask_bits).view(n, -1, CELL)
    zm = torch.where(mask, z, torch.full_like(z, MASK_FILL))
    return torch.stack([zm[..., OFFS[k]:OFFS[k + 1]].argmax(-1) for k in range(COMPS)],
                       -1).to(torch.uint8)
