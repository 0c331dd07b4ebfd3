"""GridNet layers on padded NHWC grids (ops/gridconv.py): index maps, remaps, pool, gathers
and the whole network, in the launchers' torch emulation (CPU).

With the grid dtype switched to fp32 the emulation must reproduce the nn.Module GridNet
(F.conv2d / F.max_pool2d / F.conv_transpose2d / nn.Linear) to fp32 rounding — that pins
every index map, shift, remap, pool routing and gather. tests/test_gpu_gridconv.py runs
the same launchers on the HIP kernels against this emulation."""
import copy

import pytest
import torch
import torch.nn.functional as F

from microbeast_amd.ops import gridconv as gc


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def obs_bits(n, S, seed):
    g = torch.Generator().manual_seed(seed)
    bits = torch.zeros(n, S, dtype=torch.int64)
    for off, k in [(0, 5), (5, 5), (10, 3), (13, 8), (21, 6)]:
        bits |= 1 << (off + torch.randint(0, k, (n, S), generator=g))
    return bits.to(torch.int32)


@pytest.fixture
def fp32_grids(monkeypatch):
    monkeypatch.setattr(gc, "_BF", torch.float32)


def test_phase_taps_cover_kernel_once():
    taps = [(ky, kx) for _, _, t in gc._phase_taps(5) for ky, kx, _ in t]
    assert sorted(taps) == [(ky, kx) for ky in range(3) for kx in range(3)]


def test_conv_maps_roundtrip():
    w = torch.randn(40, 27, 3, 3)
    fwd, dgrad, grad = gc.conv_maps(40, 27)
    wk = torch.where(fwd >= 0, w.reshape(-1)[fwd.long().clamp(min=0)], 0.)
    assert torch.equal(wk.view(40, 9, 32)[:, :, :27], w.permute(0, 2, 3, 1).reshape(40, 9, 27))
    assert (wk.view(40, 9, 32)[:, :, 27:] == 0).all()
    wt = torch.where(dgrad >= 0, w.reshape(-1)[dgrad.long().clamp(min=0)], 0.)
    assert torch.equal(wt.view(32, 9, 40), wk.view(40, 9, 32).permute(2, 1, 0))
    # grad map: dW laid out like wk -> back to the parameter layout
    assert torch.equal(wk.reshape(-1)[grad.long()].view_as(w), w)


def test_convt_and_critic_maps_roundtrip():
    w = torch.randn(40, 78, 3, 3)
    fwd, dgrad, grad, nfl = gc.convt_maps(40, 78)
    # a dW buffer laid out [cop, ntap*cip] per phase whose entries are the weight itself
    cip, cop = 64, 96
    buf = torch.zeros(nfl)
    off = 0
    for _, _, taps in gc._phase_taps(1):
        blk = torch.zeros(cop, len(taps), cip)
        for i, (ky, kx, _) in enumerate(taps):
            blk[:78, i, :40] = w[:, :, ky, kx].t()
        buf[off:off + blk.numel()] = blk.reshape(-1)
        off += blk.numel()
    assert torch.equal(buf[grad.long()].view_as(w), w)
    assert fwd.numel() == 78 * 9 * cip and dgrad.shape == (cip, 9 * cop)
    w1 = torch.randn(128, 256 * 2 * 3)
    fwd, dgrad, grad = gc.critic_maps(128, 256, 2, 3)
    w1p = w1.reshape(-1)[fwd.long()]
    assert torch.equal(w1p, w1.view(128, 256, 2, 3).permute(0, 2, 3, 1).reshape(128, -1))
    assert torch.equal(w1.reshape(-1)[dgrad.long()], w1p.t())
    assert torch.equal(w1p.reshape(-1)[grad.long()].view_as(w1), w1)


def test_remap_zero_border_fills_padded_convt_output():
    """the 4 phase remaps of a transposed conv with zero_border write every pixel of the
    padded output grid exactly once"""
    B, H, W = 2, 3, 4
    Hp, Wp = H + 2, W + 2
    Ho, Wo = 2 * H + 2, 2 * W + 2
    hits = torch.zeros(B * Ho * Wo, dtype=torch.int64)
    for a, b, _ in gc._phase_taps(W):
        rm = gc.remap(Hp, Wp, Ho * Wo, Wo, 2, 2, a + 1, b + 1, (Ho, Wo), True)
        _, dst, _ = gc._remap_index(B * Hp * Wp, rm, "cpu")
        hits.index_add_(0, dst, torch.ones_like(dst))
        assert gc._remap_last_row(B * Hp * Wp, rm) < B * Ho * Wo
    assert (hits == 1).all()


def test_encoder_layer_matches_conv_relu_pool(fp32_grids):
    torch.manual_seed(0)
    B, H, W, cin, cout = 3, 6, 5, 40, 64
    x = torch.randn(B, H, W, cin)
    w = (torch.randn(cout, cin, 3, 3) * 0.1).requires_grad_(True)
    b = (torch.randn(cout) * 0.1).requires_grad_(True)
    fwd, dgrad, grad = gc.conv_maps(cout, cin)
    wk = w.detach().reshape(-1)[fwd.long().clamp(min=0)] * (fwd >= 0)
    wt = w.detach().reshape(-1)[dgrad.long().clamp(min=0)] * (dgrad >= 0)
    xp = F.pad(x, (0, 64 - cin, 1, 1, 1, 1)).requires_grad_(True)
    pp, plain = gc._EncoderLayer.apply(xp, w, b, wk, wt, grad, True)
    xr = x.clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = F.max_pool2d(F.relu(F.conv2d(xr.permute(0, 3, 1, 2), wr, br, padding=1)), 3, 2, 1)
    yr = yr.permute(0, 2, 3, 1)
    assert torch.allclose(plain, yr, atol=1e-5)
    assert torch.allclose(pp[:, 1:-1, 1:-1], yr, atol=1e-5) and pp[:, 0].abs().max() == 0
    g1, g2 = torch.randn_like(pp), torch.randn_like(plain)
    ((pp * g1).sum() + (plain * g2).sum()).backward()
    (yr * (g1[:, 1:-1, 1:-1] + g2)).sum().backward()
    assert _rel(xp.grad[:, 1:-1, 1:-1, :cin], xr.grad) < 1e-5
    assert _rel(w.grad, wr.grad) < 1e-5 and _rel(b.grad, br.grad) < 1e-5


@pytest.mark.parametrize("crop,rows", [(None, None), ((5, 3), None), ((5, 3), 1)])
def test_decoder_layer_matches_conv_transpose(fp32_grids, crop, rows):
    """rows: the layer runs on that prefix of the batch (the rest gets zero input grad)"""
    torch.manual_seed(0)
    B, H, W, cin = 2, 3, 2, 64
    cout = 32 if crop is None else 78
    x = torch.randn(B, H, W, cin)
    w = (torch.randn(cin, cout, 3, 3) * 0.1).requires_grad_(True)
    b = (torch.randn(cout) * 0.1).requires_grad_(True)
    fwd, dgrad, grad, nfl = gc.convt_maps(cin, cout)
    bm = w.detach().reshape(-1)[fwd.long().clamp(min=0)] * (fwd >= 0)
    bdx = w.detach().reshape(-1)[dgrad.long().clamp(min=0)] * (dgrad >= 0)
    xp = F.pad(x, (0, 0, 1, 1, 1, 1)).requires_grad_(True)
    y = gc._DecoderLayer.apply(xp, w, b, bm, bdx, grad, crop, nfl, rows)
    if rows is not None:
        x = x[:rows]
    xr = x.clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = F.conv_transpose2d(xr.permute(0, 3, 1, 2), wr, br, stride=2, padding=1,
                            output_padding=1).permute(0, 2, 3, 1)
    if crop is None:
        yr = F.relu(yr)
        assert torch.allclose(y[:, 1:-1, 1:-1], yr, atol=1e-5) and y[:, -1].abs().max() == 0
        gy = torch.randn_like(y)
        (y * gy).sum().backward()
        (yr * gy[:, 1:-1, 1:-1]).sum().backward()
    else:
        yr = yr[:, :crop[0], :crop[1]].reshape(x.shape[0], -1)
        assert torch.allclose(y, yr, atol=1e-5)
        gy = torch.randn_like(y)
        (y * gy).sum().backward()
        (yr * gy).sum().backward()
    n = x.shape[0]
    assert _rel(xp.grad[:n, 1:-1, 1:-1], xr.grad) < 1e-5 and (xp.grad[n:] == 0).all()
    assert _rel(w.grad, wr.grad) < 1e-5 and _rel(b.grad, br.grad) < 1e-5


def test_pool_first_max_tie_rule():
    y = torch.zeros(1, 4, 4, 8, dtype=torch.bfloat16)
    y[0, 1, 1] = 1.0
    y[0, 1, 2] = 1.0      # tie inside window (0, 1) (rows -1..1, cols 1..3): pixel (1, 1)
    _, _, idx = gc.pool_fwd(y, True, False)  # = tap (ky=2, kx=0) comes first in scan order
    assert int(idx[0, 0, 1, 0]) == 2 * 3 + 0
    assert int(idx[0, 0, 0, 0]) == 2 * 3 + 2


@pytest.mark.parametrize("s", [10, 16])
def test_gridnet_grid_path_matches_module_fp32(fp32_grids, s):
    """the whole grid path (emulated, fp32 grids) == the nn.Module GridNet in fp32"""
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    m = GridNetAgent((s, s, 27))
    ref = copy.deepcopy(m)
    ref.hip_kernels = False
    ref.compute_dtype = torch.float32
    m.emulate = True
    obs = obs_bits(5, s * s, 1)
    lg, v = m.policy_value(obs)
    lr, vr = ref.policy_value(obs)
    assert lg.shape == lr.shape == (5, s * s * 78)
    assert _rel(lg, lr) < 1e-5 and _rel(v, vr) < 1e-5
    gl, gv = torch.randn(lg.shape), torch.randn(v.shape)
    ((lg * gl).sum() + (v * gv).sum()).backward()
    ((lr * gl).sum() + (vr * gv).sum()).backward()
    for (name, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) < 1e-5, name


def test_gridnet_grid_path_bf16_close():
    """bf16 grids (the GPU precision) stay close to the fp32 module"""
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
    assert lg.dtype == torch.bfloat16
    assert _rel(lg, lr) < 2e-2 and _rel(v, vr) < 2e-2


def test_direct_grads_learner_step_matches_accumulated():
    """GridNet's layers write weight gradients straight into the flat gradient slots
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
