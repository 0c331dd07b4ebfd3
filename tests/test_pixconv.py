"""GridNet on the pixel-major layout (ops/pixconv.py): pair tables, weight maps, pooling and the
whole network in the launchers' torch emulation (CPU).

With the activation dtype switched to fp32 the emulation must reproduce the nn.Module GridNet
(F.conv2d / F.max_pool2d / F.conv_transpose2d / nn.Linear) to fp32 rounding, forward and every
parameter gradient -- that pins every pair table, weight / gradient map, pool routing and
operand stride. tests/test_gpu_pixconv.py runs the same launchers on the HIP kernels."""
import copy

import pytest
import torch
import torch.nn.functional as F

from microbeast_amd.ops import cell_head
from microbeast_amd.ops import pixconv as pc


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def obs_bits(n, S, seed):
    g = torch.Generator().manual_seed(seed)
    bits = torch.zeros(n, S, dtype=torch.int64)
    for off, k in [(0, 5), (5, 5), (10, 3), (13, 8), (21, 6)]:
        bits |= 1 << (off + torch.randint(0, k, (n, S), generator=g))
    return bits.to(torch.int32)


@pytest.fixture
def fp32_acts(monkeypatch):
    monkeypatch.setattr(pc, "_BF", torch.float32)


@pytest.mark.parametrize("H,W", [(1, 1), (2, 2), (4, 3), (8, 8)])
def test_conv_pairs_are_conv2d(H, W):
    """out[P] = sum over the pair list == F.conv2d(padding=1); the dgrad and wgrad lists are
    the same (P, q, t) triples regrouped"""
    torch.manual_seed(0)
    x = torch.randn(2, 3, H, W)
    w = torch.randn(4, 3, 3, 3)
    fwd, dg, wg = pc.conv_pairs(H, W)
    xp = x.permute(2, 3, 0, 1).reshape(H * W, 2, 3)
    out = torch.zeros(H * W, 2, 4)
    for P, ents in fwd:
        for q, t in ents:
            out[P] += xp[q] @ w[:, :, t // 3, t % 3].t()
    ref = F.conv2d(x, w, padding=1).permute(2, 3, 0, 1).reshape(H * W, 2, 4)
    torch.testing.assert_close(out, ref)
    trip = sorted((P, q, t) for P, e in fwd for q, t in e)
    assert trip == sorted((P, q, t) for q, e in dg for P, t in e)
    assert trip == sorted((P, q, t) for t, e in enumerate(wg) for P, q in e)


@pytest.mark.parametrize("H,W,crop", [(1, 1, None), (2, 3, None), (8, 8, (10, 10)), (8, 8, (13, 7))])
def test_convt_pairs_are_conv_transpose2d(H, W, crop):
    torch.manual_seed(0)
    x = torch.randn(2, 3, H, W)
    w = torch.randn(3, 5, 3, 3)
    fwd, dg, wg = pc.convt_pairs(H, W, crop)
    ref = F.conv_transpose2d(x, w, stride=2, padding=1, output_padding=1)
    Ho, Wo = crop if crop else (2 * H, 2 * W)
    ref = ref[:, :, :Ho, :Wo].permute(2, 3, 0, 1).reshape(Ho * Wo, 2, 5)
    xp = x.permute(2, 3, 0, 1).reshape(H * W, 2, 3)
    out = torch.zeros(Ho * Wo, 2, 5)
    for P, ents in fwd:
        assert len(ents) in (1, 2, 4)
        for q, t in ents:
            out[P] += xp[q] @ w[:, :, t // 3, t % 3]
    torch.testing.assert_close(out, ref)
    trip = sorted((P, q, t) for P, e in fwd for q, t in e)
    assert trip == sorted((P, q, t) for q, e in dg for P, t in e)
    assert trip == sorted((P, q, t) for t, e in enumerate(wg) for P, q in e)


def test_weight_maps_roundtrip():
    w = torch.randn(40, 24, 3, 3)
    fm, dm, gm, cop = pc.conv_maps(40, 24)
    B = w.reshape(-1)[fm.long()].view(9, 40, 24)
    assert torch.equal(B, w.permute(2, 3, 0, 1).reshape(9, 40, 24))
    D = torch.where(dm >= 0, w.reshape(-1)[dm.long().clamp(min=0)], 0.).view(9, 24, cop)
    assert torch.equal(D[:, :, :40], B.transpose(1, 2)) and (D[:, :, 40:] == 0).all()
    assert torch.equal(B.reshape(-1)[gm.long()].view_as(w), w)   # dW [9][O][I] -> param
    wt = torch.randn(32, 78, 3, 3)
    fm, dm, gm = pc.convt_maps(32, 78, 96)
    B = wt.reshape(-1)[fm.long()].view(9, 78, 32)
    assert torch.equal(B, wt.permute(2, 3, 1, 0).reshape(9, 78, 32))
    D = torch.where(dm >= 0, wt.reshape(-1)[dm.long().clamp(min=0)], 0.).view(9, 32, 96)
    assert torch.equal(D[:, :, :78], B.transpose(1, 2)) and (D[:, :, 78:] == 0).all()
    dW = torch.zeros(9, 96, 32)
    dW[:, :78] = B
    assert torch.equal(dW.reshape(-1)[gm.long()].view_as(wt), wt)
    lw = torch.randn(128, 256 * 4)
    fm, dm, gm = pc.critic_maps(128, 256, 4)
    B = lw.reshape(-1)[fm.long()].view(4, 128, 256)
    assert torch.equal(B, lw.view(128, 256, 4).permute(2, 0, 1))
    assert torch.equal(lw.reshape(-1)[dm.long()].view(4, 256, 128), B.transpose(1, 2))
    assert torch.equal(B.reshape(-1)[gm.long()].view_as(lw), lw)


def test_pool_first_max_tie_rule_and_backward():
    y = torch.zeros(4 * 4, 1, 8, dtype=torch.bfloat16)
    y[1 * 4 + 1] = 1.0
    y[1 * 4 + 2] = 1.0   # tie inside window (0, 1) (rows -1..1, cols 1..3): pixel (1, 1) first
    pooled, idx = pc.ppool_fwd(y, 4, 4, 1, 8)
    assert int(idx[0 * 2 + 1, 0, 0]) == 2 * 3 + 0
    assert int(idx[0, 0, 0]) == 2 * 3 + 2
    # backward routes to the argmax only where pooled > 0 and sums overlapping windows
    g = torch.ones(4, 1, 8, dtype=torch.bfloat16)
    dy = pc.ppool_bwd(g, 1, None, 0, pooled, idx, 4, 4, 1, 8).float()
    assert dy[1 * 4 + 1, 0, 0] == 4.0      # pixel (1,1) wins windows (0,0), (0,1), (1,0), (1,1)
    assert dy.sum() == 4 * 8


@pytest.mark.parametrize("s", [10, 16, 20])
def test_gridnet_pbc_matches_module_fp32(fp32_acts, s):
    """the whole pixel-major path (emulated, fp32 activations) == the nn.Module GridNet in
    fp32: logits, value and every parameter gradient"""
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    m = GridNetAgent((s, s, 27))
    ref = copy.deepcopy(m)
    ref.hip_kernels = False
    ref.compute_dtype = torch.float32
    m.emulate = True
    n = 3
    obs = obs_bits(n, s * s, 1)
    lg, v = m.policy_value_pbc(obs)
    assert lg.shape == (s * s, n, pc.LOGIT_LD)
    lr, vr = ref.policy_value(obs)
    lgc = pc.pbc_to_cell_major(lg)
    assert lgc.shape == lr.shape == (n, s * s * 78)
    assert _rel(lgc, lr) < 1e-5 and _rel(v, vr) < 1e-5
    gl, gv = torch.randn(lr.shape), torch.randn(vr.shape)
    ((lgc * gl).sum() + (v * gv).sum()).backward()
    ((lr * gl).sum() + (vr * gv).sum()).backward()
    for (name, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) < 1e-5, name


def test_gridnet_pbc_decoder_prefix_fp32(fp32_acts):
    """n_logits: the decoder runs on the first rows only; the value (and the encoder /
    critic gradients) still cover every row"""
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(1)
    m = GridNetAgent((10, 10, 27))
    m.emulate = True
    obs = obs_bits(4, 100, 3)
    lg, v = m.policy_value_pbc(obs, 2)
    lf, vf = m.policy_value_pbc(obs)
    assert lg.shape == (100, 2, pc.LOGIT_LD) and v.shape == (4,)
    torch.testing.assert_close(pc.pbc_to_cell_major(lg), pc.pbc_to_cell_major(lf)[:2])
    torch.testing.assert_close(v, vf)


def test_gridnet_pbc_bf16_close():
    """bf16 activations (the GPU precision) stay close to the fp32 module"""
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    m = GridNetAgent((10, 10, 27))
    ref = copy.deepcopy(m)
    ref.hip_kernels = False
    ref.compute_dtype = torch.float32
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.bfloat16().float())
    m.emulate = True
    obs = obs_bits(4, 100, 2)
    lg, v = m.policy_value(obs)
    lr, vr = ref.policy_value(obs)
    assert _rel(lg, lr) < 2e-2 and _rel(v, vr) < 2e-2


def test_score_pbc_matches_cell_major():
    """scoring pixel-major logits == scoring the same logits cell-major (CPU path)"""
    torch.manual_seed(0)
    S, n = 6, 3
    lg = torch.randn(S, n, pc.LOGIT_LD, requires_grad=True)
    mask = cell_head.pack_mask(torch.rand(n, S, 78) < 0.5)
    act = torch.randint(0, 4, (n, S, 7), dtype=torch.uint8)
    lp, ent = cell_head.score_pbc(lg, mask, act)
    cm = lg.detach()[:, :, :78].permute(1, 0, 2).reshape(n, S * 78).requires_grad_(True)
    lp2, ent2 = cell_head.score(cm, mask, act)
    torch.testing.assert_close(lp, lp2)
    torch.testing.assert_close(ent, ent2)
    (lp.sum() + ent.sum()).backward()
    (lp2.sum() + ent2.sum()).backward()
    torch.testing.assert_close(lg.grad[:, :, :78].permute(1, 0, 2).reshape(n, -1), cm.grad)
    assert (lg.grad[:, :, 78:] == 0).all()


def test_direct_grads_learner_step_matches_accumulated():
    """GridNet's backward writes weight gradients straight into the flat gradient slots
    (no zero fill, no AccumulateGrad add): one learner update equals the same update with
    ordinary accumulated gradients, and every slot is adopted in place."""
    from helpers import synthetic_batch
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    base = GridNetAgent((10, 10, 27))
    base.emulate = True
    batch = synthetic_batch(base, 3, 2, 100, 0)
    outs = []
    for direct in (True, False):
        m = copy.deepcopy(base)
        for p in m.parameters():
            p._mbk_direct_grad = direct
        lr = Learner(m, LearnerHParams(), torch.device("cpu"))
        assert any(lr.flat.direct) == direct
        for _ in range(2):
            lr.learn(batch)
            assert lr.flat.adopt_grads() == 0
            assert lr.flat.check_grad_views()
        outs.append(lr.flat.data.clone())
    torch.testing.assert_close(outs[0], outs[1], rtol=0, atol=0)


def _sparse_mask(n, S, frac, seed):
    g = torch.Generator().manual_seed(seed)
    m = torch.randint(0, 2 ** 31 - 1, (n, S, 3), generator=g, dtype=torch.int32)
    m[..., 2] &= (1 << 14) - 1
    m[torch.rand(n, S, generator=g) > frac] = 0
    return m


def test_cells_compaction_order_and_maps():
    n, S = 7, 12
    mask = _sparse_mask(n, S, 0.3, 0)
    c = pc.Cells(mask, n, S)
    act = (mask != 0).any(-1)
    nact = int(act.sum())
    assert int(c.totals[0]) == nact
    cells = [int(x) for x in c.rowcell[:nact]]
    assert cells == sorted(cells, key=lambda v: (v % S, v // S))       # (cell, sample) order
    assert all(act[v // S, v % S] for v in cells)
    assert torch.equal(c.rowimg[:nact], c.rowcell[:nact] // S)
    for P in range(S):
        o, k = int(c.bucket_off[P]), int(c.bucket_cnt[P])
        assert all(int(v) % S == P for v in c.rowcell[o:o + k])
    cr = c.cellrow.view(S, n)
    for P in range(S):
        for b in range(n):
            r = int(cr[P, b])
            assert (r >= 0) == bool(act[b, P]) and (r < 0 or int(c.rowcell[r]) == b * S + P)
    assert int(c.tile_off[-1]) == int(c.totals[1])


@pytest.mark.parametrize("s", [10, 16])
def test_sparse_logits_match_dense(s):
    """scoring through the compact active-cell rows == the dense pixel-major logits layer:
    log-probs, entropies, values and every parameter gradient (emulated bf16 maths)"""
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    m = GridNetAgent((s, s, 27))
    m.emulate = True
    d = copy.deepcopy(m)
    d.sparse_logits = False
    n, ns = 6, 4
    obs = obs_bits(n, s * s, 5)
    mask = _sparse_mask(ns, s * s, 0.05, 1)
    act = torch.randint(0, 4, (ns, s * s, 7), dtype=torch.uint8)
    lp, ent, v = m.evaluate(obs, mask, act, ns)
    lq, eq, vq = d.evaluate(obs, mask, act, ns)
    torch.testing.assert_close(lp, lq)
    torch.testing.assert_close(ent, eq)
    torch.testing.assert_close(v, vq)
    (lp.sum() + 0.3 * ent.sum() + v.sum()).backward()
    (lq.sum() + 0.3 * eq.sum() + vq.sum()).backward()
    for (name, p), (_, q) in zip(m.named_parameters(), d.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-6, msg=name)


def test_sparse_act_matches_dense():
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    m = GridNetAgent((10, 10, 27))
    m.emulate = True
    d = copy.deepcopy(m)
    d.sparse_logits = False
    obs = obs_bits(5, 100, 2)
    mask = _sparse_mask(5, 100, 0.1, 3)
    a1, lp1, v1 = m.act(obs, mask, generator=torch.Generator().manual_seed(4))
    a2, lp2, v2 = d.act(obs, mask, generator=torch.Generator().manual_seed(4))
    active = (mask != 0).any(-1)
    assert torch.equal(a1[active], a2[active])
    torch.testing.assert_close(lp1, lp2)
    torch.testing.assert_close(v1, v2)


@pytest.mark.parametrize("H,crop", [(8, None), (4, None), (8, (10, 10))])
def test_pwgrad_all_equals_per_tap(H, crop):
    """the all-taps (forward-table) weight gradient == the per-tap form (emulation)"""
    torch.manual_seed(0)
    M, O, I = 40, 16, 8
    if crop is None:
        fwd, _, wg = pc.conv_pairs(H, H)
        npo = H * H
    else:
        fwd, _, wg = pc.convt_pairs(H, H, crop)
        npo = crop[0] * crop[1]
    g = torch.randn(npo * M * O)
    x = torch.randn(H * H * M * I)
    gmap = torch.arange(9 * O * I, dtype=torch.int32)
    a, b = torch.empty(9 * O * I), torch.empty(9 * O * I)
    pc.pwgrad(g, M * O, O, O, x, M * I, I, I, pc.wgrad_table(wg, "cpu"), M, gmap, a, x_relu=True)
    db = torch.empty(O)
    pc.pwgrad_all(g, M * O, O, O, x, M * I, I, I, pc.pconv_table(fwd, "cpu"), 9, M, gmap, b,
                  x_relu=True, bias_out=db)
    torch.testing.assert_close(db, g.view(-1, O).sum(0), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-4)
