"""HIP kernel numerics vs plain PyTorch fp32 references (run on the MI355X box)."""
import pytest
import torch

from microbeast_amd.ops import cell_head
from microbeast_amd.ops.cell_head import pack_mask, unpack_mask

pytestmark = pytest.mark.gpu


def _rand_cells(n, S, device, p_mask=0.35, seed=0):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(n, S * 78, generator=g) * 2.0
    mb = torch.rand(n, S, 78, generator=g) < p_mask
    # some fully masked segments and some empty cells
    mb[:, ::5, :] = False
    mb[:, 1::7, 29:78] = False
    action = torch.zeros(n, S, 7, dtype=torch.uint8)
    for k in range(7):
        o0, o1 = cell_head.OFFS[k], cell_head.OFFS[k + 1]
        w = mb[..., o0:o1].float() + 1e-9
        action[..., k] = torch.multinomial(w.view(-1, o1 - o0), 1, generator=g).view(n, S).to(torch.uint8)
    return logits.to(device), pack_mask(mb).to(device), action.to(device), mb.to(device)


def test_pack_roundtrip():
    mb = torch.rand(3, 5, 78) < 0.5
    assert torch.equal(unpack_mask(pack_mask(mb)), mb)


def test_masked_cell_score_fwd_bwd(cuda):
    n, S = 6, 64
    logits, bits, action, mb = _rand_cells(n, S, cuda)
    x = logits.clone().requires_grad_(True)
    lp, ent = cell_head.score(x, bits, action)
    xr = logits.detach().cpu().clone().requires_grad_(True)
    _, lpr, entr = cell_head.cell_head_torch(xr, mb.cpu(), action.cpu())
    torch.testing.assert_close(lp.cpu(), lpr, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(ent.cpu(), entr, rtol=1e-4, atol=1e-3)
    gl = torch.randn(n)
    ge = torch.randn(n)
    (lp * gl.to(cuda)).sum().add_((ent * ge.to(cuda)).sum()).backward()
    ((lpr * gl).sum() + (entr * ge).sum()).backward()
    torch.testing.assert_close(x.grad.cpu(), xr.grad, rtol=1e-3, atol=1e-5)


def test_masked_cell_score_bf16_logits(cuda):
    n, S = 4, 64
    logits, bits, action, mb = _rand_cells(n, S, cuda, seed=3)
    lb = logits.bfloat16()
    lp, ent = cell_head.score(lb, bits, action)
    _, lpr, entr = cell_head.cell_head_torch(lb.float().cpu(), mb.cpu(), action.cpu())
    torch.testing.assert_close(lp.cpu(), lpr, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(ent.cpu(), entr, rtol=1e-4, atol=2e-3)


def test_masked_cell_sample(cuda):
    n, S = 64, 64
    logits, bits, _, mb = _rand_cells(n, S, cuda, seed=1)
    rng = torch.tensor([1234, 0], dtype=torch.int64, device=cuda)
    a, lp = cell_head.sample(logits, bits, rng)
    assert int(rng[1].item()) == 1
    # every sampled component is legal wherever its segment has a legal entry
    for k in range(7):
        o0, o1 = cell_head.OFFS[k], cell_head.OFFS[k + 1]
        seg = mb[..., o0:o1]
        has = seg.any(-1)
        chosen = seg.gather(-1, a[..., k:k + 1].long()).squeeze(-1)
        assert bool((chosen | ~has).all())
    # logp of the samples equals scoring them
    lp2, _ = cell_head.score(logits, bits, a)
    torch.testing.assert_close(lp, lp2, rtol=1e-5, atol=1e-4)
    # sampling frequencies follow the masked softmax (one 49-way segment, many draws)
    n2 = 4096
    z = torch.randn(1, 78) * 1.5
    m = torch.zeros(1, 78, dtype=torch.bool)
    m[0, 29:78] = True
    m[0, 0] = True
    lz = z.repeat(n2, 1).to(cuda)
    bz = pack_mask(m.repeat(n2, 1).view(n2, 1, 78)).to(cuda)
    az, _ = cell_head.sample(lz, bz, rng)
    cnt = torch.bincount(az[:, 0, 6].long().cpu(), minlength=49).float() / n2
    p = torch.softmax(z[0, 29:78], 0)
    assert (cnt - p).abs().max() < 0.03


def test_vtrace_kernel_vs_torch(cuda):
    from microbeast_amd.ops.vtrace import vtrace, vtrace_torch
    T, B = 37, 300
    g = torch.Generator().manual_seed(0)
    lpn = torch.randn(T, B, generator=g) * 0.3 - 5
    lpo = lpn + torch.randn(T, B, generator=g) * 0.2
    val = torch.randn(T + 1, B, generator=g)
    rew = torch.randn(T, B, generator=g)
    done = torch.rand(T, B, generator=g) < 0.05
    ent = torch.rand(T, B, generator=g) * 3
    ref = vtrace_torch(lpn, lpo, val, rew, done, ent, reward_clip=0.0)
    out = vtrace(lpn.to(cuda), lpo.to(cuda), val.to(cuda), rew.to(cuda), done.to(cuda),
                 ent.to(cuda), want_targets=True)
    torch.testing.assert_close(out.vs.cpu(), ref.vs, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out.adv.cpu(), ref.adv, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out.g_logp.cpu(), ref.g_logp, rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(out.g_value.cpu(), ref.g_value, rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(out.losses.cpu(), ref.losses, rtol=1e-4, atol=1e-5)


def test_flat_adam_kernel_vs_torch(cuda):
    from microbeast_amd.ops.optim import FlatAdam, FlatParams
    torch.manual_seed(0)
    mc = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5))
    mg = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5)).to(cuda)
    mg.load_state_dict(mc.state_dict())
    ref = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5))
    ref.load_state_dict(mc.state_dict())
    fg = FlatParams(mg, cuda)
    ag = FlatAdam(fg, lr=1e-2, eps=1e-5, bf16_shadow=True)
    ta = torch.optim.Adam(ref.parameters(), lr=1e-2, eps=1e-5)
    for it in range(5):
        x = torch.randn(8, 33)
        fg.zero_grad()
        mg(x.to(cuda)).pow(2).sum().backward()
        ag.step()
        ta.zero_grad()
        ref(x).pow(2).sum().backward()
        ta.step()
    for p, q in zip(mg.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach().cpu(), q.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(ag.shadow.float(), fg.data, rtol=1e-2, atol=1e-2)


def test_multi_copy(cuda):
    from microbeast_amd import _native as N
    from microbeast_amd.ops.copy import multi_copy
    srcs = [torch.randint(0, 255, (n,), dtype=torch.uint8, device=cuda) for n in (1, 17, 4096, 100003)]
    dsts = [torch.zeros_like(s) for s in srcs]
    multi_copy(list(zip(srcs, dsts)))
    torch.cuda.synchronize()
    for s, d in zip(srcs, dsts):
        assert torch.equal(s, d)
    assert any("libmbk_kernels" in p for p in N.loaded_libraries())
