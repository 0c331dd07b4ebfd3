"""GridNet's HIP launchers (gemm.hip taps GEMM with remaps, fc.hip shifted wgrad, gridnet.hip
bits / pool / gather / colsum / map / value kernels) against their torch emulation
(tests/test_gridconv.py pins the emulation against F.conv2d & co. in fp32), and the whole
GridNet grid path on the GPU against the same path emulated on the CPU."""
import copy

import pytest
import torch

from test_gridconv import _rel, obs_bits
from microbeast_amd.ops import gridconv as gc

pytestmark = pytest.mark.gpu


def test_gpu_taps_gemm_remaps_match_emulation():
    torch.manual_seed(0)
    B, H, W, C, n = 3, 5, 4, 64, 78
    Hp, Wp = H + 2, W + 2
    x = torch.randn(B * Hp * Wp, C).to(torch.bfloat16)
    bm = torch.randn(n, 4 * C).to(torch.bfloat16)
    bias = torch.randn(n)
    shifts = [0, 1, Wp, Wp + 1]
    for rm, rows in [(gc.remap(Hp, Wp, 4 * H * W, 2 * W, 2, 2, 1, 0), B * 4 * H * W),
                     (gc.remap(Hp, Wp, (2 * H + 2) * (2 * W + 2), 2 * W + 2, 2, 2, 2, 1,
                               (2 * H + 2, 2 * W + 2), True), B * (2 * H + 2) * (2 * W + 2)),
                     (gc.remap(Hp, Wp, 7 * 3, 3, 2, 2, 1, 1, (7, 3)), B * 21)]:
        for dt in (torch.bfloat16, torch.float32):
            want = torch.full((rows, n), 7.0, dtype=dt)
            gc.taps_gemm([x] * 4, shifts, bm, bias, True, out=want, rm=rm)
            got = torch.full((rows, n), 7.0, dtype=dt, device="cuda")
            gc.taps_gemm([x.cuda()] * 4, shifts, bm.cuda(), bias.cuda(), True, out=got, rm=rm)
            torch.testing.assert_close(got.cpu().float(), want.float(), rtol=1e-2, atol=1e-2)


def test_gpu_taps_wgrad_matches_emulation():
    torch.manual_seed(0)
    M = 1000
    x = torch.randn(M, 64).to(torch.bfloat16)
    g = torch.randn(M, 40).to(torch.bfloat16)
    shifts = [-37, 0, 300]
    got = gc.taps_wgrad(g.cuda(), x.cuda(), shifts)
    torch.testing.assert_close(got.cpu(), gc.taps_wgrad(g, x, shifts), rtol=1e-3, atol=2e-2)


def test_gpu_bits_grid_and_pool_exact():
    torch.manual_seed(0)
    bits = obs_bits(7, 100, 3)
    want = gc.bits_grid(bits, 10, 10, 18, 18)
    got = gc.bits_grid(bits.cuda(), 10, 10, 18, 18)
    assert torch.equal(got.cpu(), want)
    y = torch.randn(5, 8, 6, 64).clamp_min(0).to(torch.bfloat16)
    y[:, 2:4, 2:4] = 0.5  # ties
    for plain, padded in ((True, True), (False, True), (True, False)):
        w = gc.pool_fwd(y, plain, padded)
        gt = gc.pool_fwd(y.cuda(), plain, padded)
        for a, b in zip(gt, w):
            assert (a is None) == (b is None)
            if a is not None:
                assert torch.equal(a.cpu(), b)
    _, pp, idx = gc.pool_fwd(y, True, True)
    g1 = torch.randn(pp.shape).to(torch.bfloat16)
    g2 = torch.randn(idx.shape).to(torch.bfloat16)
    want = gc.pool_bwd(g1, 1, g2, 0, pp, 1, idx, 8, 6)
    got = gc.pool_bwd(g1.cuda(), 1, g2.cuda(), 0, pp.cuda(), 1, idx.cuda(), 8, 6)
    torch.testing.assert_close(got.cpu().float(), want.float(), rtol=1e-2, atol=1e-2)


def test_gpu_gather_colsum_map_value_match_emulation():
    torch.manual_seed(0)
    B, H, W, C = 3, 4, 5, 40
    src = torch.randn(B, 2 * H + 2, 2 * W + 2, C).to(torch.bfloat16)
    mask = torch.randn(src.shape).to(torch.bfloat16)
    Wo = 2 * W + 2
    geo = (Wo * C + C, (2 * H + 2) * Wo * C, Wo * C, C, 2 * H, 2 * W, C)
    want = gc.grid_gather(src, geo, mask, geo[:4], 2, B, H, W, 64)
    got = gc.grid_gather(src.cuda(), geo, mask.cuda(), geo[:4], 2, B, H, W, 64)
    assert torch.equal(got.cpu(), want)
    lg = torch.randn(B, 7 * 6 * 78)  # fp32 cropped logits source
    geo = (0, 7 * 6 * 78, 6 * 78, 78, 7, 6, 78)
    want = gc.grid_gather(lg, geo, None, None, 2, B, 4, 3, 96)
    got = gc.grid_gather(lg.cuda(), geo, None, None, 2, B, 4, 3, 96)
    assert torch.equal(got.cpu(), want)
    x = torch.randn(20000, 96).to(torch.bfloat16)
    o0, o1 = torch.empty(70), torch.empty(8)
    gc.colsum(x, 78, o0, 70, o1)
    p0, p1 = torch.empty(70, device="cuda"), torch.empty(8, device="cuda")
    gc.colsum(x.cuda(), 78, p0, 70, p1)
    torch.testing.assert_close(p0.cpu(), o0, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(p1.cpu(), o1, rtol=1e-4, atol=1e-2)
    src = torch.randn(1000)
    m = torch.randint(-1, 1000, (3000,), dtype=torch.int32)
    d = torch.empty(3000, dtype=torch.bfloat16)
    gc.map_gather([(src, d, m)])
    dd = torch.empty(3000, dtype=torch.bfloat16, device="cuda")
    df = torch.empty(3000, device="cuda")
    gc.map_gather([(src.cuda(), dd, m.cuda()), (src.cuda(), df, m.cuda())])
    assert torch.equal(dd.cpu(), d)
    assert torch.equal(df.cpu().to(torch.bfloat16), d)
    dv = torch.randn(5000)
    h = torch.randn(5000, 128).clamp_min(0).to(torch.bfloat16)
    w2 = torch.randn(1, 128)
    gw, gb = torch.empty(1, 128), torch.empty(1)
    dh = gc.value_bwd(dv, h, w2, gw, gb)
    gw2, gb2 = torch.empty(1, 128, device="cuda"), torch.empty(1, device="cuda")
    dh2 = gc.value_bwd(dv.cuda(), h.cuda(), w2.cuda(), gw2, gb2)
    torch.testing.assert_close(dh2.cpu().float(), dh.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(gw2.cpu(), gw, rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(gb2.cpu(), gb, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("s", [10, 16])
def test_gpu_gridnet_matches_cpu_emulation(s):
    """the whole GridNet grid path: HIP kernels vs the same bf16 maths emulated on CPU"""
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    m = GridNetAgent((s, s, 27))
    cpu = copy.deepcopy(m)
    cpu.emulate = True
    m = m.cuda()
    obs = obs_bits(6, s * s, 1)
    lg, v = m.policy_value(obs.cuda())
    lc, vc = cpu.policy_value(obs)
    assert lg.dtype == torch.bfloat16 and lg.shape == lc.shape
    assert _rel(lg.cpu(), lc) < 1e-2 and _rel(v.cpu(), vc) < 1e-2
    gl, gv = torch.randn(lg.shape), torch.randn(v.shape)
    ((lg.float() * gl.cuda()).sum() + (v * gv.cuda()).sum()).backward()
    ((lc.float() * gl).sum() + (vc * gv).sum()).backward()
    for (name, p), (_, q) in zip(m.named_parameters(), cpu.named_parameters()):
        assert _rel(p.grad.cpu(), q.grad) < 5e-2, name
