"""Sparse per-cell action head on the HIP kernels of ``head.hip``.

Exact reformulation of the reference's dense head (actor Linear(256, 78*h*w)
+ CategoricalMasked per component, model.py:136-200): only (frame, cell)
pairs with at least one legal action are computed — a fully-masked cell has
log-prob 0, entropy 0 and zero gradient in the reference's fp32 semantics, so
skipping it changes nothing but the cost (typically 1-5 % of cells are active).

Pipeline per call: compaction (3 small launches) -> grouped MFMA GEMM with
the masked-softmax epilogue (sample or score) -> per-frame sums; backward:
per-cell recompute + dZ + dX_pair + dW_c (one workgroup per cell) -> dX gather.
"""
from __future__ import annotations


import torch

from .. import _native as N

KD, NP, NPT = 256, 80, 96


class SparseHead:
    def __init__(self, S: int, device: torch.device):
        self.S = S
        self.device = device
        self.Wp = torch.zeros(S, NP, KD, dtype=torch.bfloat16, device=device)
        self.WpT = torch.zeros(S, KD, NPT, dtype=torch.bfloat16, device=device)
        self.bp = torch.zeros(S, NP, dtype=torch.float32, device=device)
        self.totals = torch.zeros(3, dtype=torch.int32, device=device)
        self.chunk_start = torch.zeros(S, dtype=torch.int32, device=device)
        self.grp_start = torch.zeros(S, dtype=torch.int32, device=device)
        self.grp_count = torch.zeros(S, dtype=torch.int32, device=device)
        self._F = -1
        n_cu = torch.cuda.get_device_properties(device).multi_processor_count if device.type == "cuda" else 1
        self.fwd_grid = 2 * n_cu
        # acting: derive the 16-pair units from the decode's bucket counts inside head_fwd
        # (no head_units launch); False: the separate head_units kernel (reference path)
        self.count_units = True
        # learner scoring on the backward's chunk tiles (mbk_head_score: W_c staged per cell
        # run, one row per lane); False: head_fwd's 16-pair units (the tests' reference)
        self.score_tiles = True
        # the scoring forward also writes per-pair softmax statistics (lse / entropy of each
        # segment) for the backward's per-logit epilogue; it then reads the pair / chunk totals
        # (the one host sync of the head, otherwise taken by the backward). False: off (tests)
        self.score_stats = True
        self.stats = None
        self._fwd_totals = None  # (P, nch) of the batch the statistics belong to
        self._prep = None        # (mask ptr, F, abits ptr, totals) of prepare_scoring

    def _ensure(self, F: int):
        if F <= self._F:
            return
        S, dev = self.S, self.device
        fb = min(256, max(8, F // 64))  # mirrors mbk_head_fb
        nfb = (F + fb - 1) // fb
        self.cnt = torch.zeros(S * nfb, dtype=torch.int32, device=dev)
        self.off = torch.zeros(S * nfb, dtype=torch.int32, device=dev)
        self.unit_cell = torch.zeros(F * S // 16 + S + 1, dtype=torch.int32, device=dev)
        self.unit_row = torch.zeros_like(self.unit_cell)
        self.chunk_cell = torch.zeros(F * S // 512 + S + 1, dtype=torch.int32, device=dev)
        self.chunk_row = torch.zeros_like(self.chunk_cell)
        self.pairs = torch.zeros(F * S, dtype=torch.int32, device=dev)
        self.pidx = torch.zeros(F * S, dtype=torch.int32, device=dev)  # active cells only
        self.abits = torch.zeros(F * ((S + 31) // 32), dtype=torch.int32, device=dev)
        self.cell_lp = torch.zeros(F * S, dtype=torch.float32, device=dev)
        self.cell_ent = torch.zeros(F * S, dtype=torch.float32, device=dev)
        self._F = F

    # ------------------------------------------------------------ acting (bucketed) path
    def ensure_buckets(self, E: int):
        """Per-cell pair buckets filled by ``mbk_decode_obs_mask_bucket`` (acting only)."""
        self._ensure(E)
        if getattr(self, "_bucket_E", -1) != E:
            self.bucket_cnt = torch.zeros(self.S, dtype=torch.int32, device=self.device)
            self.bucket = torch.zeros(self.S * E, dtype=torch.int32, device=self.device)
            self._bucket_E = E

    def sample_bucketed(self, X: torch.Tensor, mask_bits: torch.Tensor, action: torch.Tensor,
                        rng: torch.Tensor, logp_out: torch.Tensor,
                        act16_out: torch.Tensor | None = None) -> torch.Tensor:
        """Sample with the buckets the decode kernel built this step (no sort: 3 launches).
        act16_out: also pack the actions into the env's 16-bit codes in the last launch."""
        F = X.shape[0]
        assert F == self._bucket_E
        k = N.kernels()
        st = N.stream_ptr()
        if act16_out is not None and self.count_units and self.S < 1024:
            # 2 launches: the head derives its units from the bucket counts itself, the
            # finale sums log-probs, packs the env actions and resets the counts
            N.check(k.mbk_head_fwd_counts(X.data_ptr(), self.Wp.data_ptr(), self.bp.data_ptr(),
                                          mask_bits.data_ptr(), action.data_ptr(),
                                          rng.data_ptr(), self.bucket.data_ptr(),
                                          self.bucket_cnt.data_ptr(), F, self.S, self.fwd_grid,
                                          self.cell_lp.data_ptr(), st), "head_fwd_counts")
            N.check(k.mbk_row_sum_pack(self.cell_lp.data_ptr(), F, self.S, logp_out.data_ptr(),
                                       rng.data_ptr(), action.data_ptr(), act16_out.data_ptr(),
                                       self.bucket_cnt.data_ptr(), self.S, st), "row_sum_pack")
            return logp_out
        N.check(k.mbk_head_units(self.bucket_cnt.data_ptr(), self.S, F, self.grp_start.data_ptr(),
                                 self.grp_count.data_ptr(), self.unit_cell.data_ptr(),
                                 self.unit_row.data_ptr(), self.totals.data_ptr(), st), "head_units")
        N.check(k.mbk_head_fwd(X.data_ptr(), self.Wp.data_ptr(), self.bp.data_ptr(),
                               mask_bits.data_ptr(), action.data_ptr(), rng.data_ptr(), 1,
                               self.bucket.data_ptr(), self.unit_cell.data_ptr(),
                               self.unit_row.data_ptr(), self.grp_start.data_ptr(),
                               self.grp_count.data_ptr(), self.totals.data_ptr(), self.S,
                               self.fwd_grid, self.cell_lp.data_ptr(), None, 0, st),
                "head_fwd")
        if act16_out is not None:
            N.check(k.mbk_row_sum_pack(self.cell_lp.data_ptr(), F, self.S, logp_out.data_ptr(),
                                       rng.data_ptr(), action.data_ptr(), act16_out.data_ptr(),
                                       None, 0, st), "row_sum_pack")
            return logp_out
        N.check(k.mbk_row_sum_rng(self.cell_lp.data_ptr(), F, self.S, logp_out.data_ptr(),
                                  rng.data_ptr(), st), "row_sum_rng")
        return logp_out

    def pack(self, W: torch.Tensor, b: torch.Tensor, with_t: bool):
        N.check(N.kernels().mbk_head_pack(W.data_ptr(), b.data_ptr(), self.S,
                                          self.Wp.data_ptr(), self.bp.data_ptr(),
                                          self.WpT.data_ptr() if with_t else None,
                                          N.stream_ptr()), "head_pack")

    def compact(self, mask_bits: torch.Tensor, F: int, action_zero: torch.Tensor | None,
                dense_out: bool = True, abits: torch.Tensor | None = None):
        """dense_out: zero the per-cell log-prob / entropy of inactive cells (sampling);
        scoring keeps pair-indexed outputs and sums them through pidx instead. abits: the
        frames' active-cell bitmap [F, S/32] int32 the acting step already wrote (the masks
        are then not read here); None: built from the masks."""
        self._ensure(F)
        if abits is not None:
            assert abits.is_contiguous() and abits.numel() == F * ((self.S + 31) // 32)
        self._abits = abits if abits is not None else self.abits
        N.check(N.kernels().mbk_head_compact(
            mask_bits.data_ptr(), F, self.S, self.cnt.data_ptr(), self.off.data_ptr(),
            self.grp_start.data_ptr(), self.grp_count.data_ptr(), self.unit_cell.data_ptr(),
            self.unit_row.data_ptr(), self.chunk_cell.data_ptr(), self.chunk_row.data_ptr(),
            self.chunk_start.data_ptr(), self.totals.data_ptr(), self.pairs.data_ptr(),
            self.pidx.data_ptr(), self._abits.data_ptr(), int(abits is not None),
            N.ptr(action_zero),
            self.cell_lp.data_ptr() if dense_out else None,
            self.cell_ent.data_ptr() if dense_out else None, N.stream_ptr()), "head_compact")

    def prepare_scoring(self, mask_bits: torch.Tensor, F: int, abits: torch.Tensor | None = None):
        """The scoring forward's compaction, issued before the trunk, with an asynchronous
        copy of the pair / chunk totals (which size the statistics buffer) to pinned memory:
        by the time the scoring forward reads them the trunk's kernels are queued behind the
        copy, so the head's host sync drains nothing. The next scoring ``forward`` of the same
        (mask, F, abits) skips the compaction."""
        self.compact(mask_bits, F, None, dense_out=False, abits=abits)
        ev = None
        if self.score_tiles and self.score_stats and self.totals.is_cuda:
            if getattr(self, "_tot_host", None) is None:
                self._tot_host = torch.empty(3, dtype=torch.int32, pin_memory=True)
            self._tot_host.copy_(self.totals, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self._prep = (mask_bits.data_ptr(), F, N.ptr(abits), ev)

    def forward(self, X: torch.Tensor, mask_bits: torch.Tensor, action: torch.Tensor,
                sample: bool, rng: torch.Tensor | None, logp_out: torch.Tensor | None = None,
                ent_out: torch.Tensor | None = None, want_ent: bool = True,
                abits: torch.Tensor | None = None):
        """X bf16 [F,256] contiguous. sample=True writes ``action`` (uint8 [F,S,7])."""
        F = X.shape[0]
        k = N.kernels()
        st = N.stream_ptr()
        pair_out = not sample  # scoring: pair-indexed outputs, summed per frame through pidx
        prep, self._prep = self._prep, None
        if pair_out and prep is not None and prep[:3] == (mask_bits.data_ptr(), F, N.ptr(abits)):
            pre_tot = None  # compacted by prepare_scoring; the totals are on their way
            if prep[3] is not None:
                prep[3].synchronize()
                P, _, nch = (int(v) for v in self._tot_host.tolist())
                pre_tot = (P, nch)
        else:
            prep = None
            self.compact(mask_bits, F, action if sample else None, dense_out=not pair_out,
                         abits=abits)
        self._fwd_totals = None
        if pair_out and self.score_tiles:
            stats = None
            if self.score_stats:
                if prep is not None and pre_tot is not None:
                    P, nch = pre_tot
                else:
                    P, _, nch = (int(v) for v in self.totals.tolist())
                if self.stats is None or self.stats.numel() < P * 16:
                    self.stats = torch.empty(max(P * 5 // 4, 1024) * 16, dtype=torch.float32,
                                             device=X.device)
                stats = self.stats
                self._fwd_totals = (P, nch)
            N.check(k.mbk_head_score(X.data_ptr(), self.Wp.data_ptr(), self.bp.data_ptr(),
                                     mask_bits.data_ptr(), action.data_ptr(),
                                     self.pairs.data_ptr(), self.grp_start.data_ptr(),
                                     self.grp_count.data_ptr(), self.chunk_cell.data_ptr(),
                                     self.chunk_row.data_ptr(), self.totals.data_ptr(), self.S,
                                     self.cell_lp.data_ptr(),
                                     self.cell_ent.data_ptr() if want_ent else None,
                                     N.ptr(stats), st), "head_score")
        else:
            N.check(k.mbk_head_fwd(X.data_ptr(), self.Wp.data_ptr(), self.bp.data_ptr(),
                                   mask_bits.data_ptr(), action.data_ptr(), N.ptr(rng),
                                   int(sample), self.pairs.data_ptr(), self.unit_cell.data_ptr(),
                                   self.unit_row.data_ptr(), self.grp_start.data_ptr(),
                                   self.grp_count.data_ptr(), self.totals.data_ptr(), self.S,
                                   self.fwd_grid, self.cell_lp.data_ptr(),
                                   self.cell_ent.data_ptr() if want_ent else None,
                                   int(pair_out), st), "head_fwd")
        logp = logp_out if logp_out is not None else torch.empty(F, dtype=torch.float32, device=X.device)
        ent = None
        if want_ent:
            ent = ent_out if ent_out is not None else torch.empty(F, dtype=torch.float32, device=X.device)
        if pair_out:
            N.check(k.mbk_head_pair_rowsum(self.pidx.data_ptr(), self._abits.data_ptr(), F,
                                           self.S,
                                           self.cell_lp.data_ptr(),
                                           self.cell_ent.data_ptr() if want_ent else None,
                                           logp.data_ptr(), N.ptr(ent), st), "head_pair_rowsum")
        else:
            N.check(k.mbk_row_sum(self.cell_lp.data_ptr(), F, self.S, logp.data_ptr(), st),
                    "row_sum")
            if want_ent:
                N.check(k.mbk_row_sum(self.cell_ent.data_ptr(), F, self.S, ent.data_ptr(), st),
                        "row_sum")
        if sample:
            N.check(k.mbk_rng_advance(rng.data_ptr(), st), "rng_advance")
        return logp, ent

    def backward(self, X, mask_bits, action, g_logp, g_ent, dW=None, db=None, value=None):
        """Returns (dX fp32 [F,256], dW fp32 [S*78,256], db fp32 [S*78]); dW / db may be
        given (e.g. the parameters' flat gradient slots).

        value = (dv fp32 [R], h bf16 [R, 256], wc fp32 [256], partial fp32 [parts, 257]) with
        R >= F (h's first F rows are X): instead of dX, returns the critic-fused input
        gradient dh = (dv wc + dX) * (h > 0) as bf16 [R, 256] (mbk_head_dx_value) and writes
        the critic's (dWc, dbc) partial rows for a column sum.

        Relies on the compaction left by the matching forward (same batch)."""
        F = X.shape[0]
        k = N.kernels()
        st = N.stream_ptr()
        # sizes of the pair-major dX and per-chunk dW buffers: from the scoring forward when it
        # wrote statistics for this batch, else one sync here
        fwd = self._fwd_totals
        if fwd is not None:
            P, nch = fwd
        else:
            P, _, nch = (int(v) for v in self.totals.tolist())
        dXp = torch.empty(max(P, 1), KD, dtype=torch.bfloat16, device=X.device)  # pair rows
        dWp = torch.empty(max(nch, 1), 78, KD, dtype=torch.float32, device=X.device)
        dbp = torch.empty(max(nch, 1), 78, dtype=torch.float32, device=X.device)
        if dW is None:
            dW = torch.empty(self.S * 78, KD, dtype=torch.float32, device=X.device)
        if db is None:
            db = torch.empty(self.S * 78, dtype=torch.float32, device=X.device)
        assert dW.is_contiguous() and db.is_contiguous() and dW.numel() == self.S * 78 * KD
        grid = max(1, min(nch, self.fwd_grid))  # the launcher caps it at one workgroup per CU
        N.check(k.mbk_head_bwd(X.data_ptr(), self.Wp.data_ptr(), self.WpT.data_ptr(),
                               self.bp.data_ptr(), mask_bits.data_ptr(), action.data_ptr(),
                               self.pairs.data_ptr(), self.grp_start.data_ptr(),
                               self.grp_count.data_ptr(), self.chunk_cell.data_ptr(),
                               self.chunk_row.data_ptr(), self.chunk_start.data_ptr(),
                               self.totals.data_ptr(), g_logp.data_ptr(), N.ptr(g_ent), self.S,
                               grid, dXp.data_ptr(), dWp.data_ptr(), dbp.data_ptr(),
                               dW.data_ptr(), db.data_ptr(),
                               self.stats.data_ptr() if fwd is not None else None, st),
                "head_bwd")
        if value is not None:
            dv, h, wc, partial = value
            R = h.shape[0]
            assert h.is_contiguous() and h.shape[1] == KD and dv.dtype == torch.float32
            dh = torch.empty(R, KD, dtype=torch.bfloat16, device=X.device)
            N.check(k.mbk_head_dx_value(dXp.data_ptr(), self.pidx.data_ptr(),
                                        self._abits.data_ptr(), F, self.S,
                                        dv.data_ptr(), h.data_ptr(), wc.data_ptr(), R,
                                        dh.data_ptr(), partial.data_ptr(), partial.shape[0], st),
                    "head_dx_value")
            return dh, dW, db
        dX = torch.empty(F, KD, dtype=torch.float32, device=X.device)
        N.check(k.mbk_head_dx_gather(dXp.data_ptr(), self.pidx.data_ptr(), self._abits.data_ptr(),
                                     F, self.S, dX.data_ptr(), st), "head_dx_gather")
        return dX, dW, db


class _SparseHeadScore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, W, b, mask_bits, action, head: SparseHead):
        Xc = X.contiguous()
        head.pack(W.detach(), b.detach(), with_t=True)
        logp, ent = head.forward(Xc, mask_bits, action, sample=False, rng=None)
        ctx.head = head
        ctx.save_for_backward(Xc, mask_bits, action)
        ctx.x_dtype = X.dtype
        return logp, ent

    @staticmethod
    def backward(ctx, g_logp, g_ent):
        Xc, mask_bits, action = ctx.saved_tensors
        F = Xc.shape[0]
        if g_logp is None:
            g_logp = torch.zeros(F, device=Xc.device)
        g_logp = g_logp.float().contiguous()
        g_ent = g_ent.float().contiguous() if g_ent is not None else None
        dX, dW, db = ctx.head.backward(Xc, mask_bits, action, g_logp, g_ent)
        return dX.to(ctx.x_dtype), dW, db, None, None, None


def sparse_score(X, W, b, mask_bits, action, head: SparseHead):
    """(logp [F], entropy [F]); differentiable in X, W, b."""
    return _SparseHeadScore.apply(X, W, b, mask_bits.contiguous(), action.contiguous(), head)


@torch.no_grad()
def sparse_sample(X, W, b, mask_bits, rng, head: SparseHead, action_out=None, logp_out=None,
                  prepacked: bool = False, bucketed: bool = False, act16_out=None):
    F = X.shape[0]
    if action_out is None:
        action_out = torch.empty(F, head.S, 7, dtype=torch.uint8, device=X.device)
    if not prepacked:
        head.pack(W, b, with_t=False)
    if bucketed:  # pairs were bucketed by the decode kernel (GPU actor engine)
        if logp_out is None:
            logp_out = torch.empty(F, dtype=torch.float32, device=X.device)
        return action_out, head.sample_bucketed(X.contiguous(), mask_bits.contiguous(),
                                                action_out, rng, logp_out, act16_out)
    logp, _ = head.forward(X.contiguous(), mask_bits.contiguous(), action_out, sample=True,
                           rng=rng, logp_out=logp_out, want_ent=False)
    return action_out, logp
