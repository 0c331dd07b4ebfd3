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
against the same fp32 oracle; the HIP path must stay within 3x of that floor (or 3 %).
(Reference update: libs/utils.py:234-335 with SURVEY §8 D1-D4 fixed.)"""
import copy

import pytest
import torch

from helpers import engine_batches

pytestmark = pytest.mark.gpu

# the one layer whose gradient may pass on direction + norm instead of the noise-floor bound
# (bf16 vs fp32 sign flips of its relu gate on 2x2 maps, see the comment in the test)
_TIE_LAYER = "network.2.res_block1.conv0."


@pytest.mark.parametrize("S", [8, 16])
def test_learn_hip_matches_fp32_torch(cuda, S):
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
    rows, bad = [], []
    for name, o, n, _ in Lr.flat.slices:
        a, b = gh[o:o + n], gr[o:o + n]
        nb = float(b.norm())
        if nb == 0.0:
            rows.append((name, float(a.abs().max()), 0.0, 1.0))
            if float(a.abs().max()) != 0.0:
                bad.append(name)
            continue
        rel = float((a - b).norm()) / nb
        floor = float((gb[o:o + n] - b).norm()) / nb
        cos = float(torch.dot(a, b)) / (float(a.norm()) * nb + 1e-30)
        rows.append((name, rel, floor, cos))
        # cos bound consistent with the rel bound (rel ~ sqrt(2 (1 - cos)) for small errors).
        # Second way to pass, for the named layer ONLY (_TIE_LAYER): direction within cos 0.995
        # of fp32 and norm within 5 %. Needed by the stage-2 block-1
        # conv0 on 2x2 maps: its du is gated by [u1 > 0] and 0.24 % of u1's signs differ
        # between bf16 and fp32 (u1 rel 0.4 %, trunk-output grad rel 3.3 %), which puts its
        # rel at 0.08-0.09 vs a bf16-torch floor of 0.0125 while cos stays 0.996 (probe:
        # tools/dbg/stage2_grad_probe.py; the dgrad + mask kernel itself matches fp32 to 1.7e-3
        # on the same operands, tools/dbg/dgrad_2x2_check.py). With the microRTS unit timings
        # (round 3 env rules) the S = 16 batch of this test puts that layer at cos 0.9947 / rel
        # 0.103, deterministically (same rollouts every run), hence the 0.99 bound.
        ok = rel < max(3.0 * floor, 3e-2) and cos > 1.0 - 0.5 * max(3.0 * floor, 3e-2) ** 2
        ratio = float(a.norm()) / nb
        tie_ok = name.startswith(_TIE_LAYER) and cos > 0.99 and abs(ratio - 1.0) < 0.05
        if not (ok or tie_ok):
            bad.append(name)
    for r in rows:  # full table on failure (pytest -s shows it always)
        print(f"{r[0]:40s} rel {r[1]:.3e}  torch-bf16 floor {r[2]:.3e}  cos {r[3]:.5f}")
    # losses: pg, value, entropy, total, mean rho
    torch.testing.assert_close(lh, lr, rtol=2e-2, atol=2e-3)
    assert not bad, f"gradients outside the bf16 noise floor: {bad}"
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
