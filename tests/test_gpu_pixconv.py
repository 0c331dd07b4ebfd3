"""pixconv.hip kernels (GridNet, pixel-major layout) vs the launchers' torch emulation of the
same index maths (tests/test_pixconv.py pins that emulation to F.conv2d / F.conv_transpose2d
/ F.max_pool2d), plus the pixel-major masked-cell kernels vs the cell-major ones."""
import copy

import pytest
import torch

from microbeast_amd.ops import cell_head
from microbeast_amd.ops import pixconv as pc

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def obs_bits(n, S, seed):
    g = torch.Generator().manual_seed(seed)
    bits = torch.zeros(n, S, dtype=torch.int64)
    for off, k in [(0, 5), (5, 5), (10, 3), (13, 8), (21, 6)]:
        bits |= 1 << (off + torch.randint(0, k, (n, S), generator=g))
    return bits.to(torch.int32)


@pytest.mark.parametrize("H,cin,N,layout,extras", [
    (8, 32, 64, "pbc", ()), (4, 64, 128, "pbc", ("relu",)), (2, 128, 256, "pbc", ("bias",)),
    (8, 32, 32, "nhwc", ("a_relu", "mask")), (8, 96, 32, "pbc", ("mask",)),
    (8, 32, 78, "pbc", ("bias",)), (1, 256, 128, "pbc", ("bias", "relu"))])
def test_gpu_pconv_matches_emulation(H, cin, N, layout, extras):
    torch.manual_seed(0)
    M = 300                          # not a multiple of the 128-image tile
    P = H * H
    fwd, dg, _ = pc.conv_pairs(H, H)
    tab_rows = fwd if N != 32 or "mask" not in extras else dg
    A = torch.randn(P * M * cin).to(BF)
    if layout == "pbc":
        a_ps, a_bs = M * cin, cin
        c_ps, c_bs, cld = M * max(N, 8), max(N, 8), max(N, 8)
    else:                            # image-major NHWC operands
        a_ps, a_bs = cin, P * cin
        c_ps, c_bs, cld = N, P * N, N
    if N == 78:
        c_ps, c_bs, cld = M * 96, 96, 96
    B = (torch.randn(9 * N * cin) * 0.1).to(BF)
    bias = torch.randn(N) if "bias" in extras else None
    mask = torch.randn(P * M * cld).to(BF) if "mask" in extras else None
    tab_c = pc.pconv_table(tab_rows, "cpu")
    tab_g = pc.pconv_table(tab_rows, "cuda")
    Cc = torch.zeros(P * M * cld, dtype=BF)
    Cg = torch.zeros(P * M * cld, dtype=BF, device="cuda")
    kw = dict(relu="relu" in extras, a_relu="a_relu" in extras)
    pc.pconv(A, a_ps, a_bs, cin, B, tab_c, N, M, Cc, c_ps, c_bs, bias=bias, mask=mask, **kw)
    pc.pconv(A.cuda(), a_ps, a_bs, cin, B.cuda(), tab_g, N, M, Cg, c_ps, c_bs,
             bias=None if bias is None else bias.cuda(),
             mask=None if mask is None else mask.cuda(), **kw)
    torch.cuda.synchronize()
    assert _rel(Cg.cpu(), Cc) < 1e-2
    # untouched elements stay untouched (no writes past N / M)
    if N == 78:
        assert (Cg.view(P, M, 96)[:, :, 78:] == 0).all()


@pytest.mark.parametrize("H,O,I,x_relu", [(8, 64, 32, True), (4, 128, 64, False),
                                          (2, 256, 128, False), (8, 96, 32, False)])
def test_gpu_pwgrad_matches_emulation(H, O, I, x_relu):
    torch.manual_seed(0)
    M = 700
    P = H * H
    _, _, wg = pc.conv_pairs(H, H)
    g = torch.randn(P * M * O).to(BF)
    x = torch.randn(P * M * I).to(BF)
    gmap = torch.arange(9 * O * I, dtype=torch.int32).flip(0)
    gmap[::7] = -1
    out_c = torch.empty(9 * O * I)
    out_g = torch.empty(9 * O * I, device="cuda")
    pc.pwgrad(g, M * O, O, O, x, M * I, I, I, pc.wgrad_table(wg, "cpu"), M, gmap, out_c,
              x_relu=x_relu)
    pc.pwgrad(g.cuda(), M * O, O, O, x.cuda(), M * I, I, I, pc.wgrad_table(wg, "cuda"), M,
              gmap.cuda(), out_g, x_relu=x_relu)
    torch.cuda.synchronize()
    torch.testing.assert_close(out_g.cpu(), out_c, rtol=2e-3, atol=2e-2)
    assert (out_g.cpu()[::7] == 0).all()


def test_gpu_pool_exact():
    torch.manual_seed(0)
    H, W, n, C = 8, 8, 37, 64
    y = torch.randn(H * W, n, C).clamp_min(0).to(BF)
    y[3, :, :8] = y[4, :, :8]        # ties
    pc_, ic = pc.ppool_fwd(y, H, W, n, C)
    pg, ig = pc.ppool_fwd(y.cuda(), H, W, n, C)
    assert torch.equal(pg.cpu(), pc_) and torch.equal(ig.cpu(), ic)
    g1 = torch.randn(16, n - 5, C).to(BF)
    g2 = torch.randn(16, n, C).to(BF)
    dc = pc.ppool_bwd(g1, n - 5, g2, n, pc_, ic, H, W, n, C)
    dg = pc.ppool_bwd(g1.cuda(), n - 5, g2.cuda(), n, pg, ig, H, W, n, C)
    torch.testing.assert_close(dg.cpu().float(), dc.float(), rtol=1e-2, atol=1e-2)


def test_gpu_masked_cell_pbc_matches_cell_major():
    """pixel-major scoring / sampling / backward == the cell-major kernels on the same logits"""
    torch.manual_seed(0)
    S, n = 100, 300
    lg = torch.randn(S, n, pc.LOGIT_LD, device="cuda").to(BF)
    mask = torch.randint(0, 2 ** 31 - 1, (n, S, 3), dtype=torch.int32, device="cuda")
    mask[torch.rand(n, S, device="cuda") < 0.9] = 0           # sparse active cells
    cm = lg[:, :, :78].permute(1, 0, 2).reshape(n, S * 78).contiguous()
    rng = torch.tensor([7, 3], dtype=torch.int64, device="cuda")
    a1, lp1 = cell_head.sample_pbc(lg, mask, rng.clone())
    a2, lp2 = cell_head.sample_gpu(cm, mask, rng.clone())
    assert torch.equal(a1, a2)
    torch.testing.assert_close(lp1, lp2)
    lgr = lg.clone().requires_grad_(True)
    cmr = cm.clone().requires_grad_(True)
    lp, ent = cell_head.score_pbc(lgr, mask, a1)
    lq, eq = cell_head.score(cmr, mask, a1)
    torch.testing.assert_close(lp, lq)
    torch.testing.assert_close(ent, eq)
    gl, ge = torch.randn(n, device="cuda"), torch.randn(n, device="cuda")
    ((lp * gl).sum() + (ent * ge).sum()).backward()
    ((lq * gl).sum() + (eq * ge).sum()).backward()
    d = lgr.grad
    assert (d[:, :, 78:] == 0).all()
    assert torch.equal(d[:, :, :78].permute(1, 0, 2).reshape(n, -1), cmr.grad)


@pytest.mark.parametrize("s", [10, 16])
def test_gpu_gridnet_pbc_matches_cpu_emulation(s):
    """the whole pixel-major GridNet: HIP kernels vs the same bf16 maths emulated on CPU,
    forward and every parameter gradient (the GPU's first layer runs on conv.hip)"""
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    m = GridNetAgent((s, s, 27))
    cpu = copy.deepcopy(m)
    cpu.emulate = True
    m = m.cuda()
    n = 150
    obs = obs_bits(n, s * s, 1)
    lg, v = m.policy_value_pbc(obs.cuda(), 140)
    lc, vc = cpu.policy_value_pbc(obs, 140)
    assert lg.dtype == BF and lg.shape == lc.shape == (s * s, 140, pc.LOGIT_LD)
    a, b = pc.pbc_to_cell_major(lg).cpu(), pc.pbc_to_cell_major(lc)
    assert _rel(a, b) < 1e-2 and _rel(v.cpu(), vc) < 1e-2
    gl, gv = torch.randn(a.shape), torch.randn(v.shape)
    ((pc.pbc_to_cell_major(lg) * gl.cuda()).sum() + (v * gv.cuda()).sum()).backward()
    ((pc.pbc_to_cell_major(lc) * gl).sum() + (vc * gv).sum()).backward()
    for (name, p), (_, q) in zip(m.named_parameters(), cpu.named_parameters()):
        assert _rel(p.grad.cpu(), q.grad) < 5e-2, name
