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


def _sparse_mask(n, S, frac, seed, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    m = torch.randint(0, 2 ** 31 - 1, (n, S, 3), generator=g, dtype=torch.int32)
    m[..., 2] &= (1 << 14) - 1
    m[torch.rand(n, S, generator=g) > frac] = 0
    return m.to(device)


def test_gpu_cells_compaction_matches_emulation():
    n, S = 1000, 100
    mask = _sparse_mask(n, S, 0.04, 0)
    c = pc.Cells(mask, n, S)
    g = pc.Cells(mask.cuda(), n, S)
    torch.cuda.synchronize()
    nact = int(c.totals[0])
    assert torch.equal(g.totals.cpu(), c.totals)
    for k in ("bucket_off", "bucket_cnt", "tile_off", "cellrow"):
        assert torch.equal(getattr(g, k).cpu(), getattr(c, k)), k
    assert torch.equal(g.rowimg[:nact].cpu(), c.rowimg[:nact])
    assert torch.equal(g.rowcell[:nact].cpu(), c.rowcell[:nact])


def test_gpu_sparse_pconv_pwgrad_match_emulation():
    """rows mode (logits of the active cells), gather mode (their input gradient, zero-row
    MFMA skipping) and the rows-mode weight gradient vs the torch emulation"""
    torch.manual_seed(0)
    M, S, cin = 700, 100, 32
    fwd, dg, wg = pc.convt_pairs(8, 8, (10, 10))
    mask = _sparse_mask(M, S, 0.05, 1)
    cc, cg = pc.Cells(mask, M, S), pc.Cells(mask.cuda(), M, S)
    x = torch.randn(64 * M * cin).to(BF)
    B = (torch.randn(9 * 78 * cin) * 0.1).to(BF)
    bias = torch.randn(78)
    Zc = torch.zeros(cc.cap * 96, dtype=BF)
    Zg = torch.zeros(cc.cap * 96, dtype=BF, device="cuda")
    pc.pconv(x, M * cin, cin, cin, B, pc.pconv_table(fwd, "cpu"), 78, M, Zc, 0, 96, bias=bias,
             cells=cc)
    pc.pconv(x.cuda(), M * cin, cin, cin, B.cuda(), pc.pconv_table(fwd, "cuda"), 78, M, Zg, 0, 96,
             bias=bias.cuda(), cells=cg)
    nact = int(cc.totals[0])
    a, b = Zg.view(-1, 96)[:nact, :78].cpu(), Zc.view(-1, 96)[:nact, :78]
    assert _rel(a, b) < 1e-2
    # gather-mode dgrad from compact dZ rows
    dZ = torch.randn(cc.cap * 96).to(BF)
    dZ.view(-1, 96)[:, 78:] = 0
    Bd = (torch.randn(9 * 32 * 96) * 0.1).to(BF)
    ym = torch.randn(64 * M * 32).to(BF)
    gc_ = torch.zeros(64 * M * 32, dtype=BF)
    gg = torch.zeros(64 * M * 32, dtype=BF, device="cuda")
    pc.pconv(dZ, 0, 96, 96, Bd, pc.pconv_table(dg, "cpu"), 32, M, gc_, M * 32, 32, mask=ym,
             gather=cc)
    pc.pconv(dZ.cuda(), 0, 96, 96, Bd.cuda(), pc.pconv_table(dg, "cuda"), 32, M, gg, M * 32, 32,
             mask=ym.cuda(), gather=cg)
    torch.cuda.synchronize()
    assert _rel(gg.cpu(), gc_) < 1e-2
    # rows-mode weight gradient
    gmap = torch.arange(9 * 96 * 32, dtype=torch.int32)
    wc = torch.empty(9 * 96 * 32)
    wgpu = torch.empty(9 * 96 * 32, device="cuda")
    pc.pwgrad(dZ, 0, 96, 96, x, M * cin, cin, cin, pc.wgrad_table(wg, "cpu"), M, gmap, wc,
              cells=cc)
    pc.pwgrad(dZ.cuda(), 0, 96, 96, x.cuda(), M * cin, cin, cin, pc.wgrad_table(wg, "cuda"), M,
              gmap.cuda(), wgpu, cells=cg)
    torch.cuda.synchronize()
    torch.testing.assert_close(wgpu.cpu(), wc, rtol=2e-3, atol=2e-2)
    out_c, out_g = torch.empty(78), torch.empty(78, device="cuda")
    cc.rows_colsum(dZ, 96, 78, out_c)
    cg.rows_colsum(dZ.cuda(), 96, 78, out_g)
    torch.testing.assert_close(out_g.cpu(), out_c, rtol=1e-3, atol=1e-2)


def test_gpu_masked_cell_rows_match_pbc():
    """compact-row scoring / sampling / backward == the pixel-major kernels at every active
    cell (same Philox draws), zero elsewhere"""
    torch.manual_seed(0)
    S, n = 100, 300
    lg = torch.randn(S, n, pc.LOGIT_LD, device="cuda").to(BF)
    mask = _sparse_mask(n, S, 0.08, 2, "cuda")
    cells = pc.Cells(mask, n, S)
    nact = int(cells.totals[0])
    rc = cells.rowcell[:nact].long()
    Zc = torch.zeros(cells.cap, pc.LOGIT_LD, dtype=BF, device="cuda")
    Zc[:nact] = lg.permute(1, 0, 2).reshape(n * S, -1)[rc]
    rng = torch.tensor([11, 5], dtype=torch.int64, device="cuda")
    a1, lp1 = cell_head.sample_rows(Zc, cells, mask, rng.clone())
    a2, lp2 = cell_head.sample_pbc(lg, mask, rng.clone())
    assert torch.equal(a1, a2)
    torch.testing.assert_close(lp1, lp2)
    Zr = Zc.clone().requires_grad_(True)
    lgr = lg.clone().requires_grad_(True)
    lp, ent = cell_head.score_rows(Zr, cells, mask, a1)
    lq, eq = cell_head.score_pbc(lgr, mask, a1)
    torch.testing.assert_close(lp, lq)
    torch.testing.assert_close(ent, eq)
    gl, ge = torch.randn(n, device="cuda"), torch.randn(n, device="cuda")
    ((lp * gl).sum() + (ent * ge).sum()).backward()
    ((lq * gl).sum() + (eq * ge).sum()).backward()
    d_dense = lgr.grad.permute(1, 0, 2).reshape(n * S, -1)
    assert torch.equal(Zr.grad[:nact], d_dense[rc])


@pytest.mark.parametrize("s", [10, 16])
def test_gpu_gridnet_sparse_matches_dense(s):
    """evaluate() through the active-cell rows == through the dense logits layer (GPU)"""
    from microbeast_amd.models.gridnet import GridNetAgent
    torch.manual_seed(0)
    m = GridNetAgent((s, s, 27)).cuda()
    d = copy.deepcopy(m)
    d.sparse_logits = False
    n, ns = 300, 256
    obs = obs_bits(n, s * s, 5).cuda()
    mask = _sparse_mask(ns, s * s, 0.05, 1, "cuda")
    act = torch.randint(0, 4, (ns, s * s, 7), dtype=torch.uint8, device="cuda")
    lp, ent, v = m.evaluate(obs, mask, act, ns)
    lq, eq, vq = d.evaluate(obs, mask, act, ns)
    torch.testing.assert_close(lp, lq)
    torch.testing.assert_close(ent, eq)
    torch.testing.assert_close(v, vq)
    (lp.sum() + 0.3 * ent.sum() + v.sum()).backward()
    (lq.sum() + 0.3 * eq.sum() + vq.sum()).backward()
    for (name, p), (_, q) in zip(m.named_parameters(), d.named_parameters()):
        assert _rel(p.grad, q.grad) < 1e-3, name


@pytest.mark.parametrize("H,O,I,x_relu,crop", [(8, 64, 32, True, None), (4, 128, 64, False, None),
                                                (2, 256, 128, False, None),
                                                (4, 32, 64, False, (8, 8))])
def test_gpu_pwgrad_all_matches_emulation(H, O, I, x_relu, crop):
    torch.manual_seed(0)
    M = 700
    if crop is None:
        fwd, _, _ = pc.conv_pairs(H, H)
        npo = H * H
    else:
        fwd, _, _ = pc.convt_pairs(H, H, crop)
        npo = crop[0] * crop[1]
    g = torch.randn(npo * M * O).to(BF)
    x = torch.randn(H * H * M * I).to(BF)
    gmap = torch.arange(9 * O * I, dtype=torch.int32).flip(0)
    gmap[::5] = -1
    out_c = torch.empty(9 * O * I)
    out_g = torch.empty(9 * O * I, device="cuda")
    db_c, db_g = torch.empty(O), torch.empty(O, device="cuda")
    pc.pwgrad_all(g, M * O, O, O, x, M * I, I, I, pc.pconv_table(fwd, "cpu"), 9, M, gmap, out_c,
                  x_relu=x_relu, bias_out=db_c)
    pc.pwgrad_all(g.cuda(), M * O, O, O, x.cuda(), M * I, I, I, pc.pconv_table(fwd, "cuda"), 9, M,
                  gmap.cuda(), out_g, x_relu=x_relu, bias_out=db_g)
    torch.cuda.synchronize()
    torch.testing.assert_close(out_g.cpu(), out_c, rtol=2e-3, atol=2e-2)
    torch.testing.assert_close(db_g.cpu(), db_c, rtol=1e-3, atol=1e-2)   # fused bias gradient


@pytest.mark.parametrize("cin,N,layout", [(32, 64, "nhwc_in"), (64, 32, "nhwc_out")])
def test_gpu_imgconv_matches_pconv(cin, N, layout):
    """the image-tile conv3x3 (8x8) == the per-pixel GEMM over the same conv table: GridNet
    conv2's forward (NHWC relu'd input -> pixel-major + bias + relu) and its input gradient
    (pixel-major dY, flipped weights -> NHWC, relu-masked)"""
    torch.manual_seed(0)
    M, H = 301, 8
    P = H * H
    fwd, _, _ = pc.conv_pairs(H, H)
    A = torch.randn(P * M * cin, device="cuda").to(BF)
    B = (torch.randn(9 * N * cin, device="cuda") * 0.1).to(BF)
    if layout == "nhwc_in":
        a_ps, a_bs, c_ps, c_bs = cin, P * cin, M * N, N
        kw = dict(bias=torch.randn(N, device="cuda"), relu=True, a_relu=True)
        mask = None
    else:
        a_ps, a_bs, c_ps, c_bs = M * cin, cin, N, P * N
        kw = {}
        mask = torch.randn(P * M * N, device="cuda").to(BF)
    C1 = torch.zeros(P * M * N, dtype=BF, device="cuda")
    C2 = torch.zeros(P * M * N, dtype=BF, device="cuda")
    pc.pconv(A, a_ps, a_bs, cin, B, pc.pconv_table(fwd, "cuda"), N, M, C1, c_ps, c_bs, mask=mask,
             **kw)
    pc.imgconv(A, a_ps, a_bs, cin, B, N, M, C2, c_ps, c_bs, H, mask=mask, **kw)
    torch.cuda.synchronize()
    assert _rel(C2, C1) < 1e-2


@pytest.mark.parametrize("x_layout", ["nhwc", "pbc"])
def test_gpu_imgwgrad_matches_pwgrad_all(x_layout):
    """image-tile weight gradient of the 8x8 32 -> 64 conv == the all-taps per-pixel form"""
    torch.manual_seed(0)
    M, H, O, I = 301, 8, 64, 32
    P = H * H
    fwd, _, _ = pc.conv_pairs(H, H)
    g = torch.randn(P * M * O, device="cuda").to(BF)
    x = torch.randn(P * M * I, device="cuda").to(BF)
    x_ps, x_bs = (I, P * I) if x_layout == "nhwc" else (M * I, I)
    gmap = torch.arange(9 * O * I, dtype=torch.int32, device="cuda").flip(0)
    a = torch.empty(9 * O * I, device="cuda")
    b = torch.empty(9 * O * I, device="cuda")
    pc.pwgrad_all(g, M * O, O, O, x, x_ps, x_bs, I, pc.pconv_table(fwd, "cuda"), 9, M, gmap, a,
                  x_relu=True)
    db = torch.empty(O, device="cuda")
    pc.imgwgrad(g, M * O, O, O, x, x_ps, x_bs, I, M, gmap, b, H, x_relu=True, bias_out=db)
    torch.cuda.synchronize()
    torch.testing.assert_close(b, a, rtol=2e-3, atol=2e-2)
    # fused bias gradient == fp32 per-channel sum of g (layout [P][M][O])
    torch.testing.assert_close(db, g.float().view(-1, O).sum(0), rtol=1e-3, atol=1e-2)
