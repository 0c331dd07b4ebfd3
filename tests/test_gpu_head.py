"""Sparse grouped-GEMM head (head.hip) vs the dense fp32 torch reference of the reference's
Linear(256, 78*S) + CategoricalMasked head."""
import pytest
import torch

from microbeast_amd.ops import cell_head
from microbeast_amd.ops.cell_head import pack_mask
from microbeast_amd.ops.head import SparseHead, sparse_sample, sparse_score

pytestmark = pytest.mark.gpu


def _problem(F, S, p_active=0.08, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = (torch.randn(F, 256, generator=g) * 0.5).bfloat16()
    W = torch.randn(S * 78, 256, generator=g) * 0.05
    b = torch.randn(S * 78, generator=g) * 0.1
    active = torch.rand(F, S, generator=g) < p_active
    m = (torch.rand(F, S, 78, generator=g) < 0.5) & active[..., None]
    m[..., 0] |= active  # active cells can always no-op
    a = torch.zeros(F, S, 7, dtype=torch.uint8)
    for k in range(7):
        o0, o1 = cell_head.OFFS[k], cell_head.OFFS[k + 1]
        w = m[..., o0:o1].float() + 1e-9
        a[..., k] = torch.multinomial(w.view(-1, o1 - o0), 1, generator=g).view(F, S).to(torch.uint8)
    a[~active] = 0
    return X, W, b, m, a


# (40000, 16, 0.25): ~10K pairs per cell, ~313 512-pair chunks: several 128-pair tiles per
# chunk and several chunks per workgroup of head_bwd2 (its prefetch pipeline across both)
# stats: the backward's per-logit epilogue on the scoring forward's softmax statistics (default)
# or its own per-segment reductions
@pytest.mark.parametrize("stats", [True, False])
@pytest.mark.parametrize("F,S,p", [(300, 64, 0.08), (1000, 256, 0.08), (40000, 16, 0.25)])
def test_sparse_score_fwd_bwd(cuda, F, S, p, stats):
    X, W, b, m, a = _problem(F, S, p_active=p)
    head = SparseHead(S, cuda)
    head.score_stats = stats
    Xg = X.to(cuda).requires_grad_(True)
    Wg = W.to(cuda).requires_grad_(True)
    bg = b.to(cuda).requires_grad_(True)
    lp, ent = sparse_score(Xg, Wg, bg, pack_mask(m).to(cuda), a.to(cuda), head)
    Xr = X.float().clone().requires_grad_(True)
    Wr = W.bfloat16().float().clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    logits = Xr @ Wr.T + br
    _, lpr, entr = cell_head.cell_head_torch(logits, m, a)
    torch.testing.assert_close(lp.cpu(), lpr, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(ent.cpu(), entr, rtol=1e-4, atol=2e-3)
    gl, ge = torch.randn(F), torch.randn(F)
    ((lp * gl.to(cuda)).sum() + (ent * ge.to(cuda)).sum()).backward()
    ((lpr * gl).sum() + (entr * ge).sum()).backward()
    rel = lambda x, y: ((x - y).norm() / (y.norm() + 1e-12)).item()  # noqa: E731
    assert rel(bg.grad.cpu(), br.grad) < 1e-3
    assert rel(Wg.grad.cpu(), Wr.grad) < 1e-2  # dZ rounded to bf16 for the MFMA
    assert rel(Xg.grad.float().cpu(), Xr.grad) < 1.5e-2
    # deterministic: a second identical call gives bit-identical gradients
    g1 = Wg.grad.clone()
    Wg.grad = None
    lp2, ent2 = sparse_score(Xg, Wg, bg, pack_mask(m).to(cuda), a.to(cuda), head)
    ((lp2 * gl.to(cuda)).sum() + (ent2 * ge.to(cuda)).sum()).backward()
    assert torch.equal(g1, Wg.grad)


@pytest.mark.parametrize("F,S,p", [(1000, 256, 0.08), (40000, 16, 0.25)])
def test_score_tiles_match_unit_scoring(cuda, F, S, p):
    """The learner's tiled scoring (mbk_head_score: chunk tiles, one row per lane) gives the
    per-frame log-prob / entropy of head_fwd's per-unit scoring and of the fp32 reference,
    including actions on masked logits (log-prob -1e8 - lse) and fully masked segments."""
    X, W, b, m, a = _problem(F, S, p_active=p, seed=5)
    g = torch.Generator().manual_seed(9)
    bad = (torch.rand(F, S, generator=g) < 0.05) & m.any(-1)
    a[..., 6] = torch.where(bad, torch.full_like(a[..., 6], 48), a[..., 6])  # maybe masked
    mk = pack_mask(m).to(cuda)
    outs = []
    for tiles in (True, False):
        head = SparseHead(S, cuda)
        head.score_tiles = tiles
        with torch.no_grad():
            lp, ent = sparse_score(X.to(cuda), W.to(cuda), b.to(cuda), mk, a.to(cuda), head)
        outs.append((lp.cpu(), ent.cpu()))
    logits = X.float() @ W.bfloat16().float().T + b
    _, lpr, entr = cell_head.cell_head_torch(logits, m, a)
    assert (lpr < -1e7).any()  # the masked-action path is exercised
    for lp, ent in outs:
        torch.testing.assert_close(lp, lpr, rtol=1e-4, atol=2e-3)
        torch.testing.assert_close(ent, entr, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-4)


def test_sparse_sample(cuda):
    F, S = 500, 256
    X, W, b, m, _ = _problem(F, S, seed=3)
    head = SparseHead(S, cuda)
    rng = torch.tensor([7, 0], dtype=torch.int64, device=cuda)
    mb = pack_mask(m).to(cuda)
    a, lp = sparse_sample(X.to(cuda), W.to(cuda), b.to(cuda), mb, rng, head)
    assert int(rng[1].item()) == 1
    act = m.any(-1).to(cuda)
    assert torch.all(a[~act] == 0)
    for k in range(7):
        o0, o1 = cell_head.OFFS[k], cell_head.OFFS[k + 1]
        seg = m[..., o0:o1].to(cuda)
        has = seg.any(-1)
        ok = seg.gather(-1, a[..., k:k + 1].long()).squeeze(-1) | ~has
        assert bool(ok.all())
    lp2, _ = sparse_score(X.to(cuda), W.to(cuda), b.to(cuda), mb, a, head)
    torch.testing.assert_close(lp, lp2, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("s", [16, 10])
def test_bucketed_acting_path_matches_sorted_path(cuda, s):
    """decode_obs_mask_bucket + head_units (atomic per-cell buckets) samples exactly the
    actions / log-probs of the deterministic counting-sort path (same Philox keys).
    s=16: the vectorised 16-byte zeroing of inactive envs; s=10 (S % 16 != 0): the scalar
    fallback. The action buffer is pre-filled with 9s so a missed zero store fails."""
    from microbeast_amd import _native as N
    from microbeast_amd.models.agent import Agent
    rt = N.runtime()
    E = 300
    S = s * s
    env = rt.VecEnv(s, E, 400, 2, [0, 1, 2, 3])
    env.set_validate(False)
    codes = torch.zeros(E, S, dtype=torch.int16)
    res = torch.zeros(E, dtype=torch.int32)
    rew, done = torch.zeros(E), torch.zeros(E, dtype=torch.uint8)
    env.reset(0, 0)
    g = torch.Generator().manual_seed(0)
    for _ in range(30):  # advance the games so there are many active cells
        a16 = torch.randint(0, 1 << 14, (E, S), generator=g, dtype=torch.int32).to(torch.int16)
        env.step_codes(a16.data_ptr(), codes.data_ptr(), res.data_ptr(), rew.data_ptr(),
                       done.data_ptr())
    torch.manual_seed(0)
    m = Agent((s, s, 27)).to(cuda)
    torch.nn.init.normal_(m.actor.weight, std=0.05)
    cg, rg = codes.to(cuda), res.to(cuda)
    obs = torch.empty(E, S, dtype=torch.int32, device=cuda)
    mask = torch.empty(E, S, 3, dtype=torch.int32, device=cuda)
    k = N.kernels()
    N.check(k.mbk_decode_obs_mask(cg.data_ptr(), rg.data_ptr(), E, s, s, obs.data_ptr(),
                                  mask.data_ptr(), N.stream_ptr()), "decode")
    # prepacked weights as the engine uses them; path 1 = counting-sort compaction
    m.pack_inference(cuda)
    rng1 = torch.tensor([123, 7], dtype=torch.int64, device=cuda)
    a1, lp1, v1 = m.act(obs, mask, rng1)
    head = m._head(cuda)
    head.ensure_buckets(E)
    obs2 = torch.empty_like(obs)
    mask2 = torch.empty_like(mask)
    a2 = torch.full((E, S, 7), 9, dtype=torch.uint8, device=cuda)
    lp2 = torch.empty(E, device=cuda)
    N.check(k.mbk_decode_obs_mask_bucket(cg.data_ptr(), rg.data_ptr(), E, s, s, obs2.data_ptr(),
                                         mask2.data_ptr(), head.bucket_cnt.data_ptr(),
                                         head.bucket.data_ptr(), head.cell_lp.data_ptr(),
                                         a2.data_ptr(), N.stream_ptr()), "decode_bucket")
    rng2 = torch.tensor([123, 7], dtype=torch.int64, device=cuda)
    _, _, v2 = m.act(obs2, mask2, rng2, action_out=a2, logp_out=lp2, bucketed=True)
    torch.cuda.synchronize()
    assert torch.equal(obs, obs2) and torch.equal(mask, mask2)
    active = int((mask != 0).any(-1).sum())
    assert active > 100
    assert torch.equal(a1, a2)
    torch.testing.assert_close(lp1, lp2, rtol=0, atol=0)
    torch.testing.assert_close(v1, v2, rtol=1e-2, atol=1e-2)
    assert rng1.tolist() == rng2.tolist() == [123, 8]
    assert int(head.bucket_cnt.sum()) == 0  # counters reset for the next step


def test_fused_fc_forward_matches_torch(cuda):
    """fc.hip fc_fwd: f = relu(relu(x) W5^T + b5) (bf16), v = f . wc + bc, vs fp32 torch."""
    from microbeast_amd import _native as N
    torch.manual_seed(3)
    for n, I in ((1000, 128), (77, 32), (300, 288)):
        x = torch.randn(n, I, device=cuda).bfloat16()
        w5 = (torch.randn(256, I, device=cuda) * 0.1).bfloat16()
        b5 = torch.randn(256, device=cuda) * 0.1
        wc = torch.randn(256, device=cuda) * 0.1
        bc = torch.randn(1, device=cuda)
        f = torch.empty(n, 256, dtype=torch.bfloat16, device=cuda)
        v = torch.empty(n, device=cuda)
        N.check(N.kernels().mbk_fc_fwd(x.data_ptr(), 1, w5.data_ptr(), b5.data_ptr(),
                                       wc.data_ptr(), bc.data_ptr(), n, I, 256, f.data_ptr(),
                                       v.data_ptr(), N.stream_ptr()), "fc_fwd")
        fr = torch.relu(torch.relu(x.float()) @ w5.float().t() + b5)
        vr = fr.bfloat16().float() @ wc + bc
        torch.testing.assert_close(f.float(), fr, rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(v, vr, rtol=1e-3, atol=1e-3)


def test_policy_step_fused_pack_matches_pack_kernel(cuda):
    """The policy step's last head launch (row_sum_pack) writes the env's 16-bit action codes:
    equal to pack_env_actions over the step's action bytes; the per-env log-prob equals the
    row sum of the step's per-cell log-probs."""
    from microbeast_amd import _native as N
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    s = 10
    rt = GpuActorRuntime(lambda: Agent((s, s, 27)), s, n_groups=1, envs_per_group=96, unroll=4,
                         batch_slots=1, device=cuda, n_threads=1)
    io, m = rt.io, rt.infer_model
    torch.nn.init.normal_(m.actor.weight, std=0.05)
    m.pack_inference(cuda)
    io["out_act16"].fill_(0x5555)
    rt._policy_step(io, m, rt.rng)
    torch.cuda.synchronize()
    ref = torch.empty_like(io["out_act16"])
    N.check(N.kernels().mbk_pack_env_actions(io["out_action"].data_ptr(), 96 * s * s,
                                             ref.data_ptr(), N.stream_ptr()), "pack")
    torch.cuda.synchronize()
    assert torch.equal(io["out_act16"], ref)
    head = m._head(cuda)
    lp = head.cell_lp[:96 * s * s].view(96, s * s).sum(1)
    torch.testing.assert_close(io["out_logp"], lp, rtol=1e-5, atol=1e-5)
    # same step through head_units + head_fwd + row_sum_rng + pack (counts not derived in the
    # head): identical actions, log-probs and codes from the same RNG state
    got = {k: io[k].clone() for k in ("out_action", "out_logp", "out_act16")}
    rt.rng[1] -= 1
    head.count_units = False
    try:
        rt._policy_step(io, m, rt.rng)
        torch.cuda.synchronize()
    finally:
        head.count_units = True
    for k, v in got.items():
        assert torch.equal(io[k], v), k
    assert int(head.bucket_cnt.abs().sum()) == 0  # counters reset for the next step
