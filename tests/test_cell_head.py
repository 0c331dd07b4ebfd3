"""Masked per-cell categorical head vs a literal port of the reference semantics."""
import torch
from torch.distributions.categorical import Categorical

from microbeast_amd.ops import cell_head as ch


class _RefCategoricalMasked(Categorical):
    """Behaviour of reference model.py:33-52 (CategoricalMasked)."""

    def __init__(self, logits, masks):
        self.masks = masks.bool()
        logits = torch.where(self.masks, logits, torch.tensor(-1e8))
        super().__init__(logits=logits)

    def entropy(self):
        p_log_p = self.logits * self.probs
        p_log_p = torch.where(self.masks, p_log_p, torch.tensor(0.0))
        return -p_log_p.sum(-1)


def _reference_scores(logits, mask, action, s):
    nvec = list(ch.NVEC) * (s * s)
    split_logits = torch.split(logits, nvec, dim=1)
    split_mask = torch.split(mask.reshape(logits.shape[0], -1), nvec, dim=1)
    cats = [_RefCategoricalMasked(l, m) for l, m in zip(split_logits, split_mask)]
    act = action.reshape(logits.shape[0], -1).T
    lp = torch.stack([c.log_prob(a) for a, c in zip(act, cats)]).sum(0)
    ent = torch.stack([c.entropy() for c in cats]).sum(0)
    return lp, ent


def test_score_matches_reference_loop():
    torch.manual_seed(0)
    n, s = 5, 3
    S = s * s
    logits = torch.randn(n, S * 78) * 2
    mask = torch.rand(n, S, 78) < 0.4
    mask[:, 0, :] = False          # a fully masked cell
    mask[:, 1, 29:] = False        # a fully masked segment
    action = torch.zeros(n, S, 7, dtype=torch.uint8)
    for k in range(7):
        seg = mask[..., ch.OFFS[k]:ch.OFFS[k + 1]].float() + 1e-9
        action[..., k] = torch.multinomial(seg.view(-1, seg.shape[-1]), 1).view(n, S).to(torch.uint8)
    _, lp, ent = ch.cell_head_torch(logits, mask, action)
    lpr, entr = _reference_scores(logits, mask, action.long(), s)
    torch.testing.assert_close(lp, lpr, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(ent, entr, rtol=1e-5, atol=1e-4)
    # the bit-packed mask path is identical
    _, lp2, ent2 = ch.cell_head_torch(logits, ch.pack_mask(mask), action)
    torch.testing.assert_close(lp2, lp)
    torch.testing.assert_close(ent2, ent)


def test_sampling_respects_mask_and_grad_flows():
    torch.manual_seed(1)
    n, S = 4, 16
    logits = torch.randn(n, S * 78, requires_grad=True)
    mask = torch.rand(n, S, 78) < 0.3
    a, lp, ent = ch.cell_head_torch(logits, mask, None, torch.Generator().manual_seed(0))
    for k in range(7):
        seg = mask[..., ch.OFFS[k]:ch.OFFS[k + 1]]
        has = seg.any(-1)
        ok = seg.gather(-1, a[..., k:k + 1].long()).squeeze(-1) | ~has
        assert bool(ok.all())
    (lp.sum() + ent.sum()).backward()
    g = logits.grad.view(n, S, 78)
    assert torch.all(g[~mask] == 0)  # masked logits get no gradient (torch.where)


def test_pack_unpack_and_greedy():
    mb = torch.rand(7, 11, 78) < 0.5
    assert torch.equal(ch.unpack_mask(ch.pack_mask(mb)), mb)
    logits = torch.randn(7, 11 * 78)
    g = ch.greedy(logits, ch.pack_mask(mb))
    assert g.shape == (7, 11, 7)
