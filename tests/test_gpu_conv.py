"""MFMA conv trunk (conv.hip) vs the plain PyTorch fp32 reference network."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

_WGRAD_QUEUE = 4  # common.h kQueueWgrad (off for the suite: conftest.py)


@pytest.mark.parametrize("n", [3, 700])
def test_wgrad_queue_matches_static(cuda, n):
    """The weight-gradient kernel on its work queue (16-round chunks taken by thread 0, the
    next rounds through an LDS ring) against the static stride: every round summed exactly
    once, so every parameter gradient equals the static one up to fp32 summation order."""
    from microbeast_amd import _native as N
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(5)
    m = Agent((16, 16, 27)).to(cuda)
    obs = _random_obs_bits(n, 256, seed=n + 9).to(cuda)
    m.features(obs[:1])
    enc = m._hip_enc
    params = encoder_params(m.network, 3)
    grads = {}
    for q in (0, 1):
        N.check(N.kernels().mbk_set_work_queue_site(_WGRAD_QUEUE, q), "queue site")
        for p in params:
            p.grad = None
        y = encode(obs, enc, params, True).float()
        r = torch.randn(y.shape, generator=torch.Generator().manual_seed(13)).to(cuda)
        (y * r).sum().backward()
        torch.cuda.synchronize()
        grads[q] = [p.grad.detach().clone() for p in params]
    N.check(N.kernels().mbk_set_work_queue_site(_WGRAD_QUEUE, 0), "queue site")
    assert float(grads[1][0].abs().sum()) > 0
    for i, (a, b) in enumerate(zip(grads[0], grads[1])):
        assert torch.isfinite(b).all(), i
        assert _rel_safe(b, a) < 1e-5, (i, _rel_safe(b, a))


def test_forward_work_queues_bit_identical_per_stream(cuda):
    """The learner forward's per-wave work queues (conv0_row16, res_fwd16_w88, res_blk32_wave,
    pool_conv_fwd4; common.h) against the static stride: every saved activation and the trunk
    output bit-identical, on the default stream twice (the counters reset themselves after each
    launch) and on a second stream (its own counters)."""
    from microbeast_amd import _native as N
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encoder_params
    torch.manual_seed(8)
    m = Agent((16, 16, 27)).to(cuda)
    obs = _random_obs_bits(1100, 256, seed=21).to(cuda)
    m.features(obs[:1])
    enc = m._hip_enc
    params = [p.detach() for p in encoder_params(m.network, 3)]

    def run():
        y, saved = enc.forward(obs, params, save=True)
        torch.cuda.current_stream().synchronize()
        return [t.clone() for t in saved if isinstance(t, torch.Tensor)] + [y.clone()]
    N.check(N.kernels().mbk_set_work_queues(0), "queues")
    try:
        ref = run()
    finally:
        N.check(N.kernels().mbk_set_work_queues(1), "queues")
    outs = [run(), run()]
    side = torch.cuda.Stream(cuda)
    with torch.cuda.stream(side):
        outs.append(run())
    torch.cuda.synchronize()
    for o in outs:
        assert len(o) == len(ref)
        for a, b in zip(ref, o):
            assert torch.equal(a, b)


def _rel_safe(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _random_obs_bits(n, S, seed=0):
    g = torch.Generator().manual_seed(seed)
    groups = [(0, 5), (5, 5), (10, 3), (13, 8), (21, 6)]
    bits = torch.zeros(n, S, dtype=torch.int64)
    for off, k in groups:
        idx = torch.randint(0, k, (n, S), generator=g)
        bits |= (1 << (off + idx))
    return bits.to(torch.int32)


def _rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_single_conv_layers_exact_structure(cuda):
    """One residual conv with relu-in + residual add, and one stage conv + pool, vs torch on
    bf16-rounded inputs (isolates indexing bugs from accumulated bf16 drift)."""
    from microbeast_amd.ops.encoder import HipEncoder
    torch.manual_seed(1)
    enc = HipEncoder(16, 16, 27, (16, 32, 32), cuda)
    L1 = enc.layers[1]  # 16->16 @ 8x8, relu_in
    w = torch.randn(16, 16, 3, 3) * 0.2
    b = torch.randn(16) * 0.1
    ws = [torch.randn(L.cout, L.cin_real, 3, 3) * 0.1 for L in enc.layers]
    ws[1] = w
    enc.pack([t.to(cuda).contiguous() for t in ws], with_bwd=True)
    x = torch.randn(5, 8, 8, 16).bfloat16()
    add = torch.randn(5, 8, 8, 16).bfloat16()
    y = enc._fwd(L1, x.to(cuda), b.to(cuda), add=add.to(cuda))
    xr = F.relu(x.float()).permute(0, 3, 1, 2)
    yr = F.conv2d(xr, w.bfloat16().float(), b, padding=1).permute(0, 2, 3, 1) + add.float()
    torch.testing.assert_close(y.float().cpu(), yr, rtol=2e-2, atol=2e-2)
    # dgrad of that conv: d = convT(dy) * (x > 0) + add
    dy = torch.randn(5, 8, 8, 16).bfloat16()
    d = enc._fwd(L1, dy.to(cuda), None, mask_src=x.to(cuda), add=add.to(cuda), dgrad=True)
    xt = xr.clone().requires_grad_(True)
    out = F.conv2d(xt, w.bfloat16().float(), None, padding=1)
    out.backward(dy.float().permute(0, 3, 1, 2))
    dr = xt.grad.permute(0, 2, 3, 1) * (x.float() > 0) + add.float()
    torch.testing.assert_close(d.float().cpu(), dr, rtol=2e-2, atol=3e-2)
    # wgrad of that conv
    dw = torch.zeros(16, 16, 3, 3, device=cuda)
    db = torch.zeros(16, device=cuda)
    enc._wgrad(L1, x.to(cuda), dy.to(cuda), dw, db)
    wt = w.bfloat16().float().clone().requires_grad_(True)
    bt = torch.zeros(16, requires_grad=True)
    F.conv2d(xr, wt, bt, padding=1).backward(dy.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(dw.cpu(), wt.grad, rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(db.cpu(), bt.grad, rtol=1e-2, atol=2e-2)
    # stage conv from bit planes + fused maxpool
    L0 = enc.layers[0]
    obs = _random_obs_bits(3, 256, seed=5)
    cfull = torch.empty(3, 16, 16, 16, dtype=torch.bfloat16, device=cuda)
    pidx = torch.empty(3, 8, 8, 16, dtype=torch.uint8, device=cuda)
    b0 = torch.randn(16) * 0.1
    p = enc._fwd(L0, obs.to(cuda), b0.to(cuda), y_full=cfull, pool_idx=pidx)
    from microbeast_amd.ops.obs import bits_to_planes
    planes = bits_to_planes(obs, 16, 16)
    cr = F.conv2d(planes, ws[0].bfloat16().float(), b0, padding=1)
    torch.testing.assert_close(cfull.float().cpu().permute(0, 3, 1, 2), cr, rtol=2e-2, atol=2e-2)
    pr, ir = F.max_pool2d(cfull.float().cpu().permute(0, 3, 1, 2), 3, 2, 1, return_indices=True)
    torch.testing.assert_close(p.float().cpu().permute(0, 3, 1, 2), pr, rtol=0, atol=0)
    # pool-index backward == autograd of max_pool2d
    dp = torch.randn(3, 8, 8, 16).bfloat16()
    dpg = dp.to(cuda)
    dc = torch.empty(3, 16, 16, 16, dtype=torch.bfloat16, device=cuda)
    from microbeast_amd import _native as N
    N.check(N.kernels().mbk_pool_bwd_idx(pidx.data_ptr(), dpg.data_ptr(), 3, 16, 16, 16,
                                         dc.data_ptr(), N.stream_ptr()), "pool_bwd_idx")
    ct = cfull.float().cpu().permute(0, 3, 1, 2).clone().requires_grad_(True)
    F.max_pool2d(ct, 3, 2, 1).backward(dp.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(dc.float().cpu(), ct.grad.permute(0, 2, 3, 1), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("s", [16, 24])
def test_pool_bwd_and_l0_wgrad(cuda, s):
    """pool backward vs autograd; the bit-plane layer's weight gradient (band layout on 16-
    and 24-wide maps) vs F.conv2d's"""
    from microbeast_amd import _native as N
    from microbeast_amd.ops.encoder import HipEncoder
    from microbeast_amd.ops.obs import bits_to_planes
    torch.manual_seed(2)
    # pool backward vs autograd of max_pool2d on the same bf16 values
    c = torch.randn(3, 16, 16, 16).bfloat16()
    dp = torch.randn(3, 8, 8, 16).bfloat16()
    dc = torch.empty_like(c).to(cuda)
    cg, dpg = c.to(cuda), dp.to(cuda)  # keep the device copies alive across the launch
    N.check(N.kernels().mbk_pool_bwd(cg.data_ptr(), dpg.data_ptr(), 3, 16, 16, 16,
                                     dc.data_ptr(), N.stream_ptr()), "pool_bwd")
    torch.cuda.synchronize()
    ct = c.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    F.max_pool2d(ct, 3, 2, 1).backward(dp.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(dc.float().cpu(), ct.grad.permute(0, 2, 3, 1), rtol=1e-2, atol=1e-2)
    # wgrad of the bit-plane input layer
    enc = HipEncoder(s, s, 27, (16, 32, 32), cuda)
    L0 = enc.layers[0]
    obs = _random_obs_bits(4, s * s, seed=7)
    dy = torch.randn(4, s, s, 16).bfloat16()
    dw = torch.zeros(16, 27, 3, 3, device=cuda)
    db = torch.zeros(16, device=cuda)
    enc._wgrad(L0, obs.to(cuda), dy.to(cuda), dw, db)
    planes = bits_to_planes(obs, s, s)
    wt = torch.zeros(16, 27, 3, 3, requires_grad=True)
    bt = torch.zeros(16, requires_grad=True)
    F.conv2d(planes, wt, bt, padding=1).backward(dy.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(dw.cpu(), wt.grad, rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(db.cpu(), bt.grad, rtol=1e-2, atol=2e-2)


def _bf(t):
    return t.bfloat16().float()


class _RoundBF16(torch.autograd.Function):
    """Forward: round to bf16 (what the HIP trunk stores); backward: round the gradient too."""

    @staticmethod
    def forward(ctx, x):
        return _bf(x)

    @staticmethod
    def backward(ctx, g):
        return _bf(g)


def _ref_trunk(net, planes, nst):
    """fp32 torch trunk that rounds activations / weights to bf16 where the kernels do."""
    R = _RoundBF16.apply
    x = planes
    for s in range(nst):
        cs = net[s]
        c = R(F.conv2d(x, R(cs.conv.weight), cs.conv.bias, padding=1))
        x = F.max_pool2d(c, 3, 2, 1)
        for rb in (cs.res_block0, cs.res_block1):
            u = R(F.conv2d(F.relu(x), R(rb.conv0.weight), rb.conv0.bias, padding=1))
            x = R(x + F.conv2d(F.relu(u), R(rb.conv1.weight), rb.conv1.bias, padding=1))
    return x


@pytest.mark.parametrize("s", [16, 10, 8])
def test_encoder_fwd_bwd_matches_torch(cuda, s):
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    from microbeast_amd.ops.obs import bits_to_planes
    torch.manual_seed(0)
    m = Agent((s, s, 27)).to(cuda)
    ref = copy.deepcopy(m).cpu().float()
    n = 12
    obs = _random_obs_bits(n, s * s)
    m.features(obs.to(cuda))  # builds the encoder
    params = encoder_params(m.network, 3)
    y = encode(obs.to(cuda), m._hip_enc, params, True).float()       # NHWC
    yr = _ref_trunk(ref.network, bits_to_planes(obs, s, s), 3).permute(0, 2, 3, 1)
    assert _rel(y.cpu(), yr) < 1e-2, _rel(y.cpu(), yr)
    r = torch.randn_like(yr)
    (y * r.to(cuda)).sum().backward()
    (yr * r).sum().backward()
    errs = {}
    for (name, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        if not name.startswith("network") or name.startswith("network.5"):
            continue
        assert p.grad is not None, name
        errs[name] = _rel(p.grad.cpu(), q.grad)
    print(s, max(errs.values()), errs)
    assert max(errs.values()) < 4e-2, errs


def test_deep_encoder_24x24_matches_torch(cuda):
    """4-stage trunk (impala_deep, BASELINE config 4): 20 conv layers, so the inference
    weight pack runs in several launches (<= 16 jobs each)."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    from microbeast_amd.ops.obs import bits_to_planes
    torch.manual_seed(0)
    s = 24
    m = Agent((s, s, 27), channels=(16, 32, 32, 32)).to(cuda)
    ref = copy.deepcopy(m).cpu().float()
    obs = _random_obs_bits(8, s * s)
    m.features(obs.to(cuda))
    params = encoder_params(m.network, 4)
    y = encode(obs.to(cuda), m._hip_enc, params, True).float()
    yr = _ref_trunk(ref.network, bits_to_planes(obs, s, s), 4).permute(0, 2, 3, 1)
    assert _rel(y.cpu(), yr) < 1e-2, _rel(y.cpu(), yr)
    m.pack_inference(cuda)  # 20 layers -> chunked pack launches
    with torch.no_grad():
        yp = encode(obs.to(cuda), m._hip_enc, params, False, prepacked=True).float()
    assert _rel(yp, y.detach()) < 1e-3, _rel(yp, y.detach())


def test_persistent_grid_cap_matches(cuda):
    """Capping the persistent grid makes every workgroup walk several image groups (and the
    last group partial): forward must be bit-identical, weight grads equal up to the
    partial-sum order."""
    from microbeast_amd import _native as N
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(3)
    m = Agent((16, 16, 27)).to(cuda)
    obs = _random_obs_bits(203, 256, seed=11).to(cuda)
    m.features(obs[:2])
    params = encoder_params(m.network, 3)
    r = torch.randn(203, 2, 2, 32, device=cuda)
    outs = []
    try:
        for cap in (0, 3):
            N.kernels().mbk_conv_set_grid_cap(cap)
            for p in params:
                p.grad = None
            y = encode(obs, m._hip_enc, params, True)
            (y.float() * r).sum().backward()
            outs.append((y.clone(), [p.grad.clone() for p in params]))
    finally:
        N.kernels().mbk_conv_set_grid_cap(0)
    (y0, g0), (y1, g1) = outs
    assert torch.equal(y0, y1)
    for a, b in zip(g0, g1):
        assert _rel(b.cpu(), a.cpu()) < 1e-4


def _q8(t):
    """round to OCP e4m3 (saturating) like the kernels"""
    return t.clamp(-448, 448).to(torch.float8_e4m3fn).float()


def test_fp8_conv_matches_quantized_reference(cuda):
    """One fp8 MFMA conv (relu-in + residual, and the bit-plane stage conv + pool) vs an fp32
    conv on the same e4m3-quantized operands: isolates layout / scale bugs from fp8 error."""
    from microbeast_amd.ops.encoder import HipEncoder
    from microbeast_amd.ops.obs import bits_to_planes
    torch.manual_seed(4)
    enc = HipEncoder(16, 16, 27, (16, 32, 32), cuda, fp8=True)
    ws = [torch.randn(L.cout, L.cin_real, 3, 3) * 0.1 for L in enc.layers]
    enc.pack_fp8([t.to(cuda).contiguous() for t in ws])
    scale = enc.scale8.cpu()
    so = enc._s_off
    # the per-channel scales are powers of two and the packed bytes are e4m3(w / scale)
    assert torch.all(torch.log2(scale) == torch.round(torch.log2(scale)))
    for i in (1, 6):  # res conv 16->16 @8x8, res conv 32->32 @4x4
        L = enc.layers[i]
        sc = scale[so[i]:so[i] + L.cout].view(-1, 1, 1, 1)
        wq = _q8(ws[i] / sc) * sc
        x = torch.randn(5, L.H, L.W, L.cin).bfloat16()
        add = torch.randn(5, L.H, L.W, L.cout).bfloat16()
        b = torch.randn(L.cout) * 0.1
        y = enc._fwd8(i, x.to(cuda), b.to(cuda), add=add.to(cuda))
        xr = _q8(F.relu(x.float())).permute(0, 3, 1, 2)
        yr = F.conv2d(xr, wq, b, padding=1).permute(0, 2, 3, 1) + add.float()
        torch.testing.assert_close(y.float().cpu(), yr, rtol=2e-2, atol=2e-2)
    L0 = enc.layers[0]
    obs = _random_obs_bits(3, 256, seed=6)
    b0 = torch.randn(16) * 0.1
    p = enc._fwd8(0, obs.to(cuda), b0.to(cuda))
    sc0 = scale[:16].view(-1, 1, 1, 1)
    cr = F.conv2d(bits_to_planes(obs, 16, 16), _q8(ws[0] / sc0) * sc0, b0, padding=1)
    pr = F.max_pool2d(cr.bfloat16().float(), 3, 2, 1)
    torch.testing.assert_close(p.float().cpu().permute(0, 3, 1, 2), pr, rtol=2e-2, atol=2e-2)


def test_fp8_trunk_close_to_bf16_trunk(cuda):
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(5)
    m = Agent((16, 16, 27)).to(cuda)
    obs = _random_obs_bits(64, 256, seed=8).to(cuda)
    m.features(obs[:2])
    params = encoder_params(m.network, 3)
    y16 = encode(obs, m._hip_enc, params, False).float()
    m._hip_enc.fp8 = True
    y8 = encode(obs, m._hip_enc, params, False).float()
    rel = ((y8 - y16).norm() / y16.norm()).item()
    assert rel < 0.08, rel


@pytest.mark.parametrize("s", [16, 10, 8])
def test_fused_fp8_trunk_matches_per_layer_fp8_kernels(cuda, s):
    """trunk.hip trunk_tail8 (fp8 layers 1..14 in one launch, e4m3 LDS tiles, bf16 residual
    stream) == the 14 per-layer fp8 MFMA conv launches: same conversion points, scales and
    fp32 accumulation order -> bit-identical."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(17)
    m = Agent((s, s, 27)).to(cuda)
    obs = _random_obs_bits(203, s * s, seed=19).to(cuda)
    m.features(obs[:2])
    enc = m._hip_enc
    params = encoder_params(m.network, 3)
    enc.fp8 = True
    assert enc.fused_tail and enc.fused_tail8
    y_fused = encode(obs, enc, params, False)
    enc.fused_tail8 = False
    y_ref = encode(obs, enc, params, False)
    enc.fused_tail8 = True
    enc.fp8 = False
    assert y_fused.shape == y_ref.shape
    assert torch.equal(y_fused, y_ref), (y_fused.float() - y_ref.float()).abs().max()


@pytest.mark.parametrize("s", [16, 10, 8])
def test_fused_trunk_tail_matches_per_layer_kernels(cuda, s):
    """trunk.hip (layers 1..14 in one launch, LDS-resident) == the per-layer conv kernels."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(7)
    m = Agent((s, s, 27)).to(cuda)
    obs = _random_obs_bits(203, s * s, seed=9).to(cuda)
    m.features(obs[:2])
    enc = m._hip_enc
    params = encoder_params(m.network, 3)
    assert enc.fused_tail
    y_fused = encode(obs, enc, params, False)
    enc.fused_tail = False
    y_ref = encode(obs, enc, params, False)
    enc.fused_tail = True
    assert y_fused.shape == y_ref.shape
    # same bf16 storage points and fp32 accumulation order per pixel -> bit-identical
    assert torch.equal(y_fused, y_ref), (y_fused.float() - y_ref.float()).abs().max()


@pytest.mark.parametrize("H,W,C", [(16, 16, 16), (8, 8, 32), (5, 5, 32), (3, 3, 32), (10, 10, 16),
                                   (12, 12, 32), (6, 6, 32)])
def test_pool_bwd_idx_shapes(cuda, H, W, C):
    """Stored-argmax pool backward on odd / even maps and both channel widths vs autograd."""
    from microbeast_amd import _native as N
    torch.manual_seed(H * 100 + C)
    n = 7
    c = torch.randn(n, C, H, W).bfloat16().float()
    pr, ir = F.max_pool2d(c, 3, 2, 1, return_indices=True)
    Ho, Wo = pr.shape[2:]
    # flat input index -> tap id ky*3+kx of the window (oy, ox)
    iy, ix = ir // W, ir % W
    oy = torch.arange(Ho).view(1, 1, Ho, 1)
    ox = torch.arange(Wo).view(1, 1, 1, Wo)
    tap = ((iy - (2 * oy - 1)) * 3 + (ix - (2 * ox - 1))).to(torch.uint8)
    pidx = tap.permute(0, 2, 3, 1).contiguous().to(cuda)
    dp = torch.randn(n, Ho, Wo, C).bfloat16()
    dpg = dp.to(cuda)
    dc = torch.empty(n, H, W, C, dtype=torch.bfloat16, device=cuda)
    N.check(N.kernels().mbk_pool_bwd_idx(pidx.data_ptr(), dpg.data_ptr(), n, H, W, C,
                                         dc.data_ptr(), N.stream_ptr()), "pool_bwd_idx")
    torch.cuda.synchronize()
    ct = c.clone().requires_grad_(True)
    F.max_pool2d(ct, 3, 2, 1).backward(dp.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(dc.float().cpu(), ct.grad.permute(0, 2, 3, 1), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("n,pool,cout,s", [(203, True, 16, 16), (7, True, 16, 16),
                                            (9, False, 16, 16), (203, True, 32, 16),
                                            (9, False, 32, 16), (41, True, 16, 24),
                                            (9, False, 16, 24), (11, True, 16, 20),
                                            (37, True, 32, -16)])
def test_conv0_row_kernel_bit_identical_to_generic(cuda, n, pool, cout, s):
    """The 16-wide stage-0 conv (register row window + DPP pixel shifts) runs the MFMA taps
    in the generic kernel's order: outputs, pre-pool values and argmax bytes are identical.
    cout 32 is GridNet's first layer (two 16-channel blocks per expanded fragment); s 24 / 20:
    the WIDE form (16-column blocks whose edge neighbours come from the next block's word,
    BASELINE config 4's 24x24 maps); s -16: a 10x10 map zero-padded to 16x16 (GridNet's first
    layer), whose all-zero row windows skip their MFMAs."""
    padded = s < 0
    s = abs(s)
    from microbeast_amd import _native as N
    from microbeast_amd.ops.encoder import HipEncoder
    torch.manual_seed(3)
    enc = HipEncoder(s, s, 27, (cout, 32, 32), cuda)
    ws = [torch.randn(L.cout, L.cin_real, 3, 3, device=cuda) * 0.2 for L in enc.layers]
    enc.pack(ws, with_bwd=False)
    L0 = enc.layers[0]
    obs = _random_obs_bits(n, s * s, seed=n).to(cuda)
    if padded:
        obs.view(n, s, s)[:, 10:] = 0
        obs.view(n, s, s)[:, :, 10:] = 0
    so = (s + 1) // 2
    b0 = torch.randn(cout, device=cuda) * 0.1
    outs = []
    for on in (1, 0):
        N.kernels().mbk_conv0_row_set(on)
        try:
            if pool:
                cfull = torch.full((n, s, s, cout), 7.0, dtype=torch.bfloat16, device=cuda)
                pidx = torch.full((n, so, so, cout), 255, dtype=torch.uint8, device=cuda)
                p = enc._fwd(L0, obs, b0, y_full=cfull, pool_idx=pidx)
                outs.append((p, cfull, pidx))
            else:  # raw launch without the pool (the encoder always pools stage convs)
                from microbeast_amd.ops.encoder import _imgs_fwd
                y = torch.empty(n, s, s, cout, dtype=torch.bfloat16, device=cuda)
                imgs = _imgs_fwd(L0, L0.cin, L0.cout, True, False)  # the generic kernel's tile
                N.check(N.kernels().mbk_conv_fwd(
                    obs.data_ptr(), 1, L0.cin, L0.cout, enc.packed_fwd.data_ptr() + 2 * L0.w_off,
                    b0.data_ptr(), 0, 0, y.data_ptr(), 0, 0, n, s, s, imgs, 0, 0,
                    N.stream_ptr()), "conv_fwd")
                outs.append((y,))
        finally:
            N.kernels().mbk_conv0_row_set(1)
    torch.cuda.synchronize()
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
    if not pool:
        from microbeast_amd.ops.obs import bits_to_planes
        cr = F.conv2d(bits_to_planes(obs.cpu(), s, s), ws[0].cpu().bfloat16().float(), b0.cpu(),
                      padding=1)
        torch.testing.assert_close(outs[0][0].float().cpu().permute(0, 3, 1, 2), cr, rtol=2e-2,
                                   atol=2e-2)


@pytest.mark.parametrize("s,n", [(16, 37), (10, 21), (24, 5)])
def test_fused_res_bwd16_matches_per_layer_kernels(cuda, s, n):
    """resblock.hip (one launch per 16-channel residual block backward) against the four
    per-layer kernels: the input gradients flowing on are bit-identical (same MFMA chains,
    same bf16 rounding), so the stage conv's grads are too; the residual-block weight grads
    differ only by fp32 summation order."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(1)
    chans = (16, 32, 32, 32) if s == 24 else (16, 32, 32)
    m = Agent((s, s, 27), channels=chans).to(cuda)
    obs = _random_obs_bits(n, s * s).to(cuda)
    m.features(obs)
    enc = m._hip_enc
    params = encoder_params(m.network, len(chans))
    grads = {}
    for fused in (False, True):
        enc.fused_res_bwd = fused
        for p in params:
            p.grad = None
        y = encode(obs, enc, params, True).float()
        r = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).to(cuda)
        (y * r).sum().backward()
        torch.cuda.synchronize()
        grads[fused] = [p.grad.detach().clone() for p in params]
    for i, (a, b) in enumerate(zip(grads[False], grads[True])):
        if i < 2:  # stage conv (weight, bias): downstream of bit-identical dp
            assert torch.equal(a, b), i
        else:
            torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("n", [1, 5, 37, 700])
def test_pool_conv_bwd_stage1_matches_per_layer(cuda, n):
    """stagebwd.hip (pool backward + weight gradient + input gradient of the 16 -> 32 stage
    conv on 8x8 maps, and of the 32 -> 32 stage conv on 4x4 maps, each in one launch; odd n:
    a stage-2 image pair's lone last image) against pool_bwd_idx + conv_wgrad + the conv_fwd
    dgrad:
    the input gradient and everything upstream of it agree to bf16 rounding of the dc sums
    (identical whenever the <= 4 windows of a pixel sum exactly in fp32), the stage conv's
    weight / bias gradients to fp32 summation order."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(3)
    m = Agent((16, 16, 27)).to(cuda)
    obs = _random_obs_bits(n, 256, seed=n + 1).to(cuda)
    m.features(obs[:1])
    enc = m._hip_enc
    params = encoder_params(m.network, 3)
    grads = {}
    for fused in (False, True):
        enc.fused_pool_conv_bwd = fused
        for p in params:
            p.grad = None
        y = encode(obs, enc, params, True).float()
        r = torch.randn(y.shape, generator=torch.Generator().manual_seed(9)).to(cuda)
        (y * r).sum().backward()
        torch.cuda.synchronize()
        grads[fused] = [p.grad.detach().clone() for p in params]
    enc.fused_pool_conv_bwd = True
    for i, (a, b) in enumerate(zip(grads[False], grads[True])):
        assert torch.isfinite(b).all(), i
        torch.testing.assert_close(b, a, rtol=2e-3, atol=1e-5, msg=f"param {i}")
    # stage 2's residual blocks run before both fused launches: untouched
    for i in range(22, 30):
        assert torch.equal(grads[False][i], grads[True][i]), i


@pytest.mark.parametrize("n", [1, 2, 37, 300])
def test_pool_fused_stage0_wgrad_matches(cuda, n):
    """The observation layer's weight gradient with the max-pool backward scattered into its
    own LDS staging (conv.hip UNPOOL, 16-wide maps) against pool_bwd_idx + the band-layout
    kernel: the same dY tile up to one bf16 rounding where two windows chose the same pixel,
    the same MFMA chains and partial rows; the other layers' gradients are untouched."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(2)
    m = Agent((16, 16, 27)).to(cuda)
    obs = _random_obs_bits(n, 256, seed=n).to(cuda)
    m.features(obs[:1])
    enc = m._hip_enc
    params = encoder_params(m.network, 3)
    grads = {}
    for fused in (False, True):
        enc.fused_pool_wgrad0 = fused
        for p in params:
            p.grad = None
        y = encode(obs, enc, params, True).float()
        r = torch.randn(y.shape, generator=torch.Generator().manual_seed(7)).to(cuda)
        (y * r).sum().backward()
        torch.cuda.synchronize()
        grads[fused] = [p.grad.detach().clone() for p in params]
    enc.fused_pool_wgrad0 = True
    assert float(grads[True][0].abs().sum()) > 0
    for i, (a, b) in enumerate(zip(grads[False], grads[True])):
        if i < 2:
            rel = float((b - a).norm() / a.norm())
            assert rel < 5e-3, (i, rel, float((b - a).abs().max()), float(a.abs().max()))
        else:
            assert torch.equal(a, b), i


@pytest.mark.parametrize("n,fused", [(5, True), (700, True), (37, False)])
def test_batched_deferred_reduce_bit_identical(cuda, n, fused):
    """One mbk_wgrad_reduce_batch launch pair at the end of the backward pass (conv.hip) against
    a reduce per layer right after its kernel: the same adds in the same order -> every
    parameter gradient bit-identical (n=700: two-level reduces; fused=False: the per-layer
    conv_wgrad path)."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(4)
    m = Agent((16, 16, 27)).to(cuda)
    obs = _random_obs_bits(n, 256, seed=n + 3).to(cuda)
    m.features(obs[:1])
    enc = m._hip_enc
    params = encoder_params(m.network, 3)
    enc.fused_res_bwd = enc.fused_res_bwd32 = fused
    grads = {}
    for defer in (False, True):
        enc.defer_reduce = defer
        for p in params:
            p.grad = None
        y = encode(obs, enc, params, True).float()
        r = torch.randn(y.shape, generator=torch.Generator().manual_seed(11)).to(cuda)
        (y * r).sum().backward()
        torch.cuda.synchronize()
        grads[defer] = [p.grad.detach().clone() for p in params]
    enc.fused_res_bwd = enc.fused_res_bwd32 = enc.defer_reduce = True
    assert float(grads[True][0].abs().sum()) > 0
    for i, (a, b) in enumerate(zip(grads[False], grads[True])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("s,n", [(16, 37), (10, 21)])
def test_fused_res_fwd16_bit_identical(cuda, s, n):
    """resblock.hip res_fwd16 (both 16-channel residual blocks in one launch) writes the
    same u0 / y0 / u1 / y1 bits as four conv_fwd launches."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encoder_params
    torch.manual_seed(2)
    m = Agent((s, s, 27)).to(cuda)
    obs = _random_obs_bits(n, s * s).to(cuda)
    m.features(obs)
    enc = m._hip_enc
    params = [p.detach() for p in encoder_params(m.network, 3)]
    outs = {}
    for fused in (False, True):
        enc.fused_res_fwd = fused
        y, saved = enc.forward(obs, params, save=True)
        torch.cuda.synchronize()
        outs[fused] = [t.clone() for t in saved[:6]] + [y.clone()]
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("s,n", [(16, 37), (10, 21), (24, 9)])
def test_fused_stage_conv_in_res_fwd16_bit_identical(cuda, s, n):
    """res_fwd16_stage (the stage-0 residual kernel also runs stage 1's conv 16->32 + max-pool
    from LDS) writes the same pooled output and argmax bytes, and every other saved
    activation, as the separate pooled conv_fwd launch."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encoder_params
    torch.manual_seed(6)
    chans = (16, 32, 32, 32) if s == 24 else (16, 32, 32)
    m = Agent((s, s, 27), channels=chans).to(cuda)
    obs = _random_obs_bits(n, s * s, seed=3).to(cuda)
    m.features(obs)
    enc = m._hip_enc
    params = [p.detach() for p in encoder_params(m.network, len(chans))]
    outs = {}
    for fused in (False, True):
        enc.fused_stage_fwd = fused
        y, saved = enc.forward(obs, params, save=True)
        torch.cuda.synchronize()
        outs[fused] = [t.clone() for t in saved if torch.is_tensor(t)] + [y.clone()]
    enc.fused_stage_fwd = True
    assert len(outs[False]) == len(outs[True])
    for i, (a, b) in enumerate(zip(outs[False], outs[True])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("s,n", [(16, 37), (14, 21), (16, 1), (16, 1001)])
def test_pool_conv_fwd4_bit_identical(cuda, s, n):
    """stage2.hip (the 32 -> 32 stage conv + max-pool on 4x4 maps, wave-owned images) writes
    the same pooled output and argmax bytes as the pooled conv_fwd launch; every other saved
    activation and the trunk output follow (odd n: a pair's lone last image)."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encoder_params
    torch.manual_seed(8)
    m = Agent((s, s, 27)).to(cuda)
    obs = _random_obs_bits(n, s * s, seed=5).to(cuda)
    m.features(obs)
    enc = m._hip_enc
    params = [p.detach() for p in encoder_params(m.network, 3)]
    outs = {}
    for fused in (False, True):
        enc.fused_pool_fwd4 = fused
        y, saved = enc.forward(obs, params, save=True)
        torch.cuda.synchronize()
        outs[fused] = [t.clone() for t in saved if torch.is_tensor(t)] + [y.clone()]
    enc.fused_pool_fwd4 = True
    assert len(outs[False]) == len(outs[True])
    for i, (a, b) in enumerate(zip(outs[False], outs[True])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("s,n", [(16, 1), (16, 3), (16, 37), (16, 1002), (14, 21)])
def test_res_blk32_wave_bit_identical(cuda, s, n):
    """The wave-owned 32-channel residual blocks (4x4 maps: one image per 16-pixel block; 2x2
    maps: image quads; no workgroup barriers) write the same u and y as the round-based
    res_blk32 kernel (n % 4 != 0: a partial last quad; 14x14: 4x4 and 2x2 stage maps)."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encoder_params
    torch.manual_seed(9)
    m = Agent((s, s, 27)).to(cuda)
    obs = _random_obs_bits(n, s * s, seed=7).to(cuda)
    m.features(obs)
    enc = m._hip_enc
    params = [p.detach() for p in encoder_params(m.network, 3)]
    outs = {}
    for fused in (False, True):
        enc.fused_res_blk32_wave = fused
        y, saved = enc.forward(obs, params, save=True)
        torch.cuda.synchronize()
        outs[fused] = [t.clone() for t in saved if torch.is_tensor(t)] + [y.clone()]
    enc.fused_res_blk32_wave = True
    for i, (a, b) in enumerate(zip(outs[False], outs[True])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("s,n", [(16, 37), (10, 21), (24, 9)])
def test_fused_res_blk32_bit_identical(cuda, s, n):
    """resblock.hip res_blk32 (one 32-channel residual block per launch, weights of both
    layers in registers) writes the same bits for every saved activation as the per-layer
    conv_fwd path."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encoder_params
    torch.manual_seed(3)
    m = Agent((s, s, 27)).to(cuda)
    obs = _random_obs_bits(n, s * s).to(cuda)
    m.features(obs)
    enc = m._hip_enc
    params = [p.detach() for p in encoder_params(m.network, 3)]
    outs = {}
    for fused in (False, True):
        enc.fused_res_fwd32 = fused
        y, saved = enc.forward(obs, params, save=True)
        torch.cuda.synchronize()
        outs[fused] = [t.clone() for t in saved if torch.is_tensor(t)] + [y.clone()]
    assert len(outs[False]) == len(outs[True])
    for i, (a, b) in enumerate(zip(outs[False], outs[True])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("s,n", [(16, 1), (16, 3), (16, 37), (16, 1001), (14, 21)])
def test_res_bwd32_team_matches_round_kernel(cuda, s, n):
    """The wave-team backward of the 32-channel blocks on 4x4 / 2x2 maps (stager + dW1, du, dx,
    dW0 waves on 32-pixel items, LDS flags) against the round-based res_bwd32 kernel: every
    input gradient flowing on is bit-identical (same dgrad chains), so every other layer's
    gradients are too; the teams' residual weight gradients differ by fp32 summation order
    (n = 1, 3: a partial last item)."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(5)
    m = Agent((s, s, 27)).to(cuda)
    obs = _random_obs_bits(n, s * s, seed=n).to(cuda)
    m.features(obs)
    enc = m._hip_enc
    params = encoder_params(m.network, 3)
    grads = {}
    for team in (False, True):
        enc.fused_res_bwd32_team = team
        for p in params:
            p.grad = None
        y = encode(obs, enc, params, True).float()
        r = torch.randn(y.shape, generator=torch.Generator().manual_seed(8)).to(cuda)
        (y * r).sum().backward()
        torch.cuda.synchronize()
        grads[team] = [p.grad.detach().clone() for p in params]
    enc.fused_res_bwd32_team = True
    for i, (a, b) in enumerate(zip(grads[False], grads[True])):
        layer = i // 2
        assert torch.isfinite(b).all(), i
        if layer >= 5 and layer % 5 != 0:  # 32-channel residual conv
            torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-6, msg=f"param {i}")
        else:
            assert torch.equal(a, b), i


@pytest.mark.parametrize("s,n", [(16, 37), (10, 21), (24, 9)])
def test_fused_res_bwd32_matches_per_layer_kernels(cuda, s, n):
    """resblock.hip res_bwd32 (one 8-wave launch per 32-channel residual block backward)
    against the per-layer wgrad / dgrad kernels: input gradients flowing on are
    bit-identical (same dgrad MFMA chains and bf16 rounding), so every non-residual weight
    gradient is too; the 32-channel residual weight grads differ by fp32 summation order."""
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import encode, encoder_params
    torch.manual_seed(4)
    chans = (16, 32, 32, 32) if s == 24 else (16, 32, 32)
    m = Agent((s, s, 27), channels=chans).to(cuda)
    obs = _random_obs_bits(n, s * s).to(cuda)
    m.features(obs)
    enc = m._hip_enc
    params = encoder_params(m.network, len(chans))
    grads = {}
    for fused in (False, True):
        enc.fused_res_bwd32 = fused
        for p in params:
            p.grad = None
        y = encode(obs, enc, params, True).float()
        r = torch.randn(y.shape, generator=torch.Generator().manual_seed(6)).to(cuda)
        (y * r).sum().backward()
        torch.cuda.synchronize()
        grads[fused] = [p.grad.detach().clone() for p in params]
    enc.fused_res_bwd32 = True
    for i, (a, b) in enumerate(zip(grads[False], grads[True])):
        layer = i // 2
        if layer >= 5 and layer % 5 != 0:  # 32-channel residual conv
            torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-6)
        else:
            assert torch.equal(a, b), i
