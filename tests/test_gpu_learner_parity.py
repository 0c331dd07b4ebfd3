"""Whole-update parity of the flagship GPU learner against an independent fp32 oracle.

One ``Learner.learn`` on the HIP path — bit-plane obs -> conv.hip trunk (bf16 MFMA, fused
pool / relu / residual) -> NHWC-permuted network.5 (gemm.hip) -> sparse head (head.hip) ->
vtrace.hip -> hand-written backward -> adam.hip — against the same update computed by the
pure-PyTorch path in fp32 on the CPU (nn.Conv2d / max_pool2d / dense Linear head / masked
categoricals / V-trace recurrence in torch ops / torch Adam math), from the same initial
weights on the same rollout batch (real GPU-engine rollouts, off-policy by one update).
Compared: the 5 losses, every parameter's gradient, and the post-Adam parameters.
The gradient tolerance is the bf16 noise floor measured on the same update: the PyTorch
path run on the GPU under bf16 autocast (MIOpen / hipBLASLt, a different implementation)
against the same fp32 oracle, and for the residual blocks' conv0 layers the spread that
rounding-level flips of their relu gate cause (their weight gradients are sums with heavy
cancellation: tests/test_relu_flip_conditioning.py); the HIP path must stay within 3x of that
floor (or 3 %). The residual conv0 layers are split operand-swap style: the HIP
gradient against the oracle's operands gated by HIP's own u is held to that same 3x floor, and
the gate itself must be no noisier than torch-bf16's (relative error of u) and flip signs only
at rounding-level |u| (within 4x torch-bf16's 99th-percentile deviation).

The gate's effect on dW. Per-flip attribution (_flip_attribution, printed
with -s): a flip at (n, co, y, x) adds or removes the rank-1 term du * relu(x)-patch to dW[co],
so a gate's effect is bounded by the sum of |du| |patch| over its flips. On this test's
deterministic update (12 residual conv0 layers over S = 8 and 16):
  * the input patch norms at the flips equal the layer's mean for HIP and torch-bf16 alike
    (the flips are not where activity is high);
  * |du| is heavy-tailed, and a gate's dW effect is set by the few flips that land on its
    tail: mean |du| at the flips ranges 0.25-5x the layer mean for HIP and 0.1-2.8x for torch;
  * torch-bf16's own gate moves dW by up to 8.0 % (network.1.res_block0 at S = 8), HIP's by
    up to 11.2 % (network.1.res_block0 / network.2.res_block1 at S = 16);
  * averaged over a map size's 6 layers: S = 8 (generic residual kernels) HIP 0.5 % vs torch
    2.8 %; S = 16 (the wave-owned w88 / 32-channel wave kernels) HIP 6.2 % vs torch 1.8 %. At
    S = 16 HIP's flips sit at 3-5x the layer's mean |du| in 4 of 6 layers while its u is still
    2-3x closer to fp32 than torch's: the flips are as few and as small in |u| as torch's, but
    land on larger-gradient positions. That correlation is measured, not explained.
The round-5 "7.7 % vs 0.3 %" was one such layer. The gate part is capped at 15 % per layer
(from 25 %; measured max 11.2 %) and, per map size, at 4x the independent bf16
implementation's mean effect (measured 3.4x at S = 16), so a kernel change that moves HIP's
gate further from bf16 behaviour fails. No layer has an escape clause.
(Reference update: libs/utils.py:234-335 with SURVEY §8 D1-D4 fixed.)"""
import copy

import numpy as np
import pytest
import torch

from helpers import engine_batches

pytestmark = pytest.mark.gpu



def _gate_hooks(model):
    """Capture every residual block's conv0 operands in the fp32 oracle: block input x, conv0
    output u (the relu gate of its gradient), block-output gradient g, conv1's pre-update
    weight."""
    caps = {}
    for si in range(len(model.channels)):
        for bi in (0, 1):
            blk = getattr(model.network[si], f"res_block{bi}")
            c = caps.setdefault(f"network.{si}.res_block{bi}.conv0.", {})
            c["w1"] = blk.conv1.weight.detach().double().clone()
            blk.register_forward_pre_hook(lambda m, i, c=c: c.__setitem__("x", i[0].detach()))
            blk.conv0.register_forward_hook(lambda m, i, o, c=c: c.__setitem__("u", o.detach()))
            def out_hook(m, i, o, c=c):  # (a forward hook's return value replaces the output)
                o.register_hook(lambda g, c=c: c.__setitem__("g", g.detach()))
            blk.register_forward_hook(out_hook)
    return caps


def _conv0_grads(c, w0, gate_u):
    """fp64 (weight, bias) gradient of a residual block's conv0 from the fp32 oracle's own
    operands (block input x, block-output gradient g, conv1 weight) with the relu gate
    [gate_u > 0] of its choice."""
    import torch.nn.functional as F
    x, g = c["x"].double(), c["g"].double()
    du = torch.nn.grad.conv2d_input(c["u"].shape, c["w1"], g, padding=1) * (gate_u > 0)
    return (torch.nn.grad.conv2d_weight(F.relu(x), tuple(w0.shape), du, padding=1),
            du.sum((0, 2, 3)))


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


def _flip_attribution(c, u_r, u_gate, ref_w):
    """Per-flip attribution of a gate's effect on a residual conv0's weight gradient: a flip at
    (n, co, y, x) adds or removes the rank-1 term du[n, co, y, x] * relu(x)[n, :, y-1..y+1,
    x-1..x+1] to dW[co]; its size is |du| times the norm of that input patch. Returns the flips'
    summed term norms and their largest one (both relative to |dW_ref|), the mean |du| at the
    flips against the mean |du| over the layer, and the gate's measured effect on dW."""
    import torch.nn.functional as F
    x, g = c["x"].double(), c["g"].double()
    du = torch.nn.grad.conv2d_input(c["u"].shape, c["w1"], g, padding=1)  # ungated
    xr = F.relu(x)
    pn = F.avg_pool2d((xr * xr).sum(1, keepdim=True), 3, 1, 1, count_include_pad=True) * 9.0
    pn = pn.sqrt()  # |patch| at every output position [N, 1, H, W]
    flips = (u_gate > 0) != (u_r > 0)
    term = (du.abs() * pn)[flips]
    nw = float(ref_w.norm()) + 1e-30
    w_gate, _ = _conv0_grads(c, c["w0"], u_gate)
    pfl = pn.expand_as(du)[flips]
    return {"flips": int(flips.sum()), "sum_term": float(term.sum()) / nw,
            "patch_at_flip": float(pfl.mean()) if pfl.numel() else 0.0,
            "patch_mean": float(pn.mean()),
            "max_term": (float(term.max()) / nw) if term.numel() else 0.0,
            "du_at_flip": float(du.abs()[flips].mean()) if term.numel() else 0.0,
            "du_mean": float(du.abs().mean()), "dW_rel": _rel(w_gate, ref_w)}


def _hip_gates(monkeypatch):
    """Capture the HIP path's own residual conv0 outputs (u0, u1 of every stage, NHWC bf16)
    as its backward reads them."""
    from microbeast_amd.ops import encoder as E
    caps = {}
    orig = E.HipEncoder.backward

    def bwd(self, g, saved, params):
        for s in range(len(saved) // 6):
            _x, _pidx, _p, u0, _y0, u1 = saved[6 * s:6 * s + 6]
            caps[f"network.{s}.res_block0.conv0."] = u0.detach().float().cpu()
            caps[f"network.{s}.res_block1.conv0."] = u1.detach().float().cpu()
        return orig(self, g, saved, params)

    monkeypatch.setattr(E.HipEncoder, "backward", bwd)
    return caps


@pytest.mark.parametrize("S", [8, 16])
def test_learn_hip_matches_fp32_torch(cuda, S, monkeypatch):
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent

    # 4 x 64 envs x T=8 = 512 frames per slot: a 128-frame batch let single max-pool argmax
    # ties (bf16 vs fp32 routing of a pooled gradient) swing one layer's relative error past
    # 3x the floor in ~1 of 5 runs
    batches = engine_batches(cuda, S, 2, groups=4, envs=64, T=8, seed=S)
    b_gpu = batches[1]  # behaviour policy = learner after one update: rho != 1 somewhere
    torch.manual_seed(7)
    base = Agent((S, S, 27))
    # the reference initialises the actor with gain 0 (all-zero weights); give it small
    # random weights so the head's forward and the dX path carry signal in this test
    with torch.no_grad():
        base.actor.weight.normal_(0, 0.02)
        base.actor.bias.normal_(0, 0.02)
    hip_model = copy.deepcopy(base)
    ref_model = copy.deepcopy(base)
    ref_model.hip_kernels = False
    ref_model.compute_dtype = torch.float32
    bf_model = copy.deepcopy(base)
    bf_model.hip_kernels = False  # torch ops under bf16 autocast on the GPU
    hp = LearnerHParams()
    caps = _gate_hooks(ref_model)
    w0s = {n: p.detach().clone() for n, p in ref_model.named_parameters() if n.endswith("conv0.weight")}
    hip_u = _hip_gates(monkeypatch)
    u_bf = {}  # torch-bf16 conv0 outputs: an independent bf16 implementation's relu gates
    for si in range(len(bf_model.channels)):
        for bi in (0, 1):
            cv = getattr(bf_model.network[si], f"res_block{bi}").conv0
            cv.register_forward_hook(lambda m, i, o, k=f"network.{si}.res_block{bi}.conv0.":
                                     u_bf.__setitem__(k, o.detach().float().cpu()))
    Lh = Learner(hip_model, hp, cuda)
    Lr = Learner(ref_model, hp, torch.device("cpu"))
    Lb = Learner(bf_model, hp, cuda)
    assert torch.equal(Lh.flat.data.cpu(), Lr.flat.data)
    lh = Lh.learn(b_gpu).cpu()
    lr = Lr.learn({k: v.cpu() for k, v in b_gpu.items()})
    Lb.learn(b_gpu)
    torch.cuda.synchronize()
    gb = Lb.flat.grad.cpu()
    print(f"losses hip {lh.tolist()}\nlosses ref {lr.tolist()}")
    gh, gr = Lh.flat.grad.cpu(), Lr.flat.grad
    # residual conv0 layers, operand-swap split: the HIP gradient against the
    # oracle's own operands gated by HIP's u (the rest: held to the ordinary bf16 floor), and that
    # gate's effect against the bf16-rounding gate-noise floor (capped), separately
    split = {}
    for pre, c in caps.items():
        n = c["u"].shape[0]
        u_h = hip_u[pre][:n].permute(0, 3, 1, 2).double()
        w0 = w0s[pre + "weight"]
        c["w0"] = w0
        ref_w, ref_b = _conv0_grads(c, w0, c["u"].double())
        hg_w, hg_b = _conv0_grads(c, w0, u_h)
        # the gate itself: HIP's u must be no noisier than an independent bf16 implementation's
        # (torch under autocast) and flip signs only at rounding-level |u|; its effect on dW is
        # then chance (these sums are ill-conditioned in the gate: tools/dbg/gate_flips.py,
        # tests/test_relu_flip_conditioning.py) and is only capped
        u_r, u_b = c["u"].double(), u_bf[pre][:n].double()
        dev = (u_b - u_r).abs().flatten()
        dev99 = float(torch.quantile(dev[torch.randperm(dev.numel(),
                                                        generator=torch.Generator().manual_seed(0))[:1 << 20]],
                                     0.99))
        flips = (u_h > 0) != (u_r > 0)
        gate = {"u_rel": _rel(u_h, u_r), "u_rel_bf": _rel(u_b, u_r), "flips": int(flips.sum()),
                "max_u_at_flip": float(u_r[flips].abs().max()) if bool(flips.any()) else 0.0,
                "dev99": dev99,
                "attr_hip": _flip_attribution(c, u_r, u_h, ref_w),
                "attr_bf": _flip_attribution(c, u_r, u_b, ref_w)}
        split[pre + "weight"] = (hg_w.float().flatten(), _rel(hg_w, ref_w), gate)
        split[pre + "bias"] = (hg_b.float(), _rel(hg_b, ref_b), gate)
    rows, bad = [], []
    gate_effects = []  # (HIP, torch-bf16) gate effect on each residual conv0's dW
    for name, o, n, _ in Lr.flat.slices:
        a, b = gh[o:o + n], gr[o:o + n]
        nb = float(b.norm())
        if nb == 0.0:
            rows.append((name, float(a.abs().max()), 0.0, 1.0, ""))
            if float(a.abs().max()) != 0.0:
                bad.append(name)
            continue
        rel = float((a - b).norm()) / nb
        # the bf16 floor of this layer: an independent bf16 implementation (torch under
        # autocast) on the same update against the same oracle; the HIP path stays within 3x
        floor = float((gb[o:o + n] - b).norm()) / nb
        cos = float(torch.dot(a, b)) / (float(a.norm()) * nb + 1e-30)
        tol = max(3.0 * floor, 3e-2)
        note = ""
        if name in split:  # residual conv0: the rest (HIP vs its own gate) and the gate part
            ref_gate, gate_rel, gt = split[name]
            rest = float((a - ref_gate).norm()) / (float(ref_gate.norm()) + 1e-30)
            gate_ok = (gt["u_rel"] <= 1.5 * gt["u_rel_bf"] + 1e-6
                       and gt["max_u_at_flip"] <= 4.0 * gt["dev99"] and gate_rel < 0.15)
            if name.endswith("weight"):  # (the bias row shares the layer's gate)
                gate_effects.append((gt["attr_hip"]["dW_rel"], gt["attr_bf"]["dW_rel"]))
            ok = rest < tol and gate_ok
            ah, ab = gt["attr_hip"], gt["attr_bf"]
            note = (f"  rest {rest:.3e} (tol {tol:.2e})  gate: dW {gate_rel:.3e}, u rel "
                    f"{gt['u_rel']:.2e} (bf16 {gt['u_rel_bf']:.2e}), {gt['flips']} flips at "
                    f"|u| <= {gt['max_u_at_flip']:.2e} (4 x bf16 dev99 {4 * gt['dev99']:.2e})"
                    f"\n      flip attribution hip: {ah['flips']} flips, sum |du||patch| "
                    f"{ah['sum_term']:.3e}, max {ah['max_term']:.3e}, |du| at flips "
                    f"{ah['du_at_flip']:.2e} vs mean {ah['du_mean']:.2e}, |patch| at flips "
                    f"{ah['patch_at_flip']:.2e} vs mean {ah['patch_mean']:.2e}, dW {ah['dW_rel']:.3e}"
                    f"\n      flip attribution bf16: {ab['flips']} flips, sum |du||patch| "
                    f"{ab['sum_term']:.3e}, max {ab['max_term']:.3e}, |du| at flips "
                    f"{ab['du_at_flip']:.2e} vs mean {ab['du_mean']:.2e}, |patch| at flips "
                    f"{ab['patch_at_flip']:.2e} vs mean {ab['patch_mean']:.2e}, dW {ab['dW_rel']:.3e}")
        else:
            ok = rel < tol and cos > 1.0 - 0.5 * tol ** 2  # (rel ~ sqrt(2 (1 - cos)))
        rows.append((name, rel, floor, cos, note))
        if not ok:
            bad.append(name)
    for r in rows:  # full table (pytest -s shows it; the floors are printed and pinned here)
        print(f"{r[0]:40s} rel {r[1]:.3e}  bf16 floor {r[2]:.3e}  cos {r[3]:.5f}{r[4]}")
    # losses: pg, value, entropy, total, mean rho
    torch.testing.assert_close(lh, lr, rtol=2e-2, atol=2e-3)
    assert not bad, f"gradients outside the bf16 noise floor: {bad}"
    # the HIP gate is not systematically worse than an independent bf16 implementation's
    gh_mean = float(np.mean([h for h, _ in gate_effects]))
    gb_mean = float(np.mean([b for _, b in gate_effects]))
    print(f"gate effect on residual conv0 dW, mean over layers: hip {gh_mean:.3e} "
          f"torch-bf16 {gb_mean:.3e}")
    assert gh_mean <= 4.0 * gb_mean + 1e-4, (gh_mean, gb_mean)
    # Adam's first step is ~lr * sign(g): equal except where a tiny gradient flips sign
    d = (Lh.flat.data.cpu() - Lr.flat.data).abs()
    assert float(d.max()) <= 2.0 * hp.lr + 1e-6
    assert float((d > 0.5 * hp.lr).float().mean()) < 0.02


def test_fused_dx_value_matches_separate_kernels(cuda):
    """head.hip head_dx_value (head dX gather + critic backward in one pass, bf16 dh) gives
    the same update as head_dx_gather (fp32 dX) + gridnet.hip value_bwd."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops import tail

    batches = engine_batches(cuda, 16, 1, envs=32, T=8, seed=3)
    torch.manual_seed(5)
    base = Agent((16, 16, 27))
    with torch.no_grad():
        base.actor.weight.normal_(0, 0.02)
    grads = []
    for fused in (True, False):
        tail._FUSED_DX_VALUE = fused
        try:
            L = Learner(copy.deepcopy(base), LearnerHParams(), cuda)
            L.learn(batches[0])
            torch.cuda.synchronize()
            grads.append((L.flat.grad.cpu().clone(), L.flat.slices))
        finally:
            tail._FUSED_DX_VALUE = True
    (ga, slices), (gb, _) = grads
    for name, o, n, _ in slices:
        a, b = ga[o:o + n], gb[o:o + n]
        scale = float(b.abs().max()) + 1e-12
        assert float((a - b).abs().max()) <= 1e-3 * scale + 1e-7, name
