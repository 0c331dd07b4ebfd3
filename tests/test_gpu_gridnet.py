"""GridNet on the pixel-major HIP kernels (ops/pixconv.py) vs the same model's PyTorch
path (fp32 reference with bf16-rounded weights): logits, value and gradients."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _obs_bits(n, S, seed):
    g = torch.Generator().manual_seed(seed)
    bits = torch.zeros(n, S, dtype=torch.int64)
    for off, k in [(0, 5), (5, 5), (10, 3), (13, 8), (21, 6)]:
        bits |= 1 << (off + torch.randint(0, k, (n, S), generator=g))
    return bits.to(torch.int32)


@pytest.mark.parametrize("s", [10, 16])
def test_gridnet_hip_matches_torch(cuda, s):
    from microbeast_amd.models.gridnet import GridNetAgent
    from microbeast_amd.ops.cell_head import OFFS, unpack_mask
    torch.manual_seed(0)
    m = GridNetAgent((s, s, 27)).to(cuda)
    ref = copy.deepcopy(m).float()
    ref.hip_kernels = False
    ref.compute_dtype = torch.float32
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.bfloat16().float())
    n = 24
    obs = _obs_bits(n, s * s, 1).to(cuda)
    lg, v = m.policy_value(obs)
    lr, vr = ref.policy_value(obs)
    assert lg.shape == lr.shape == (n, s * s * 78)
    assert _rel(lg, lr) < 3e-2, _rel(lg, lr)
    assert _rel(v, vr) < 3e-2, _rel(v, vr)
    # gradients through evaluate (masked-cell scoring of sampled actions)
    mask = torch.randint(0, 2 ** 31 - 1, (n, s * s, 3), dtype=torch.int32, device=cuda)
    mask[..., 2] &= (1 << 14) - 1
    a, _, _ = m.act(obs, mask, torch.tensor([1, 0], dtype=torch.int64, device=cuda))
    logp, ent, val = m.evaluate(obs, mask, a)
    (logp.sum() + 0.1 * ent.sum() + val.sum()).backward()
    logp_r, ent_r, val_r = ref.evaluate(obs, mask, a)
    (logp_r.sum() + 0.1 * ent_r.sum() + val_r.sum()).backward()
    errs = {name: _rel(p.grad, q.grad) for (name, p), (_, q) in
            zip(m.named_parameters(), ref.named_parameters()) if p.grad is not None}
    assert len(errs) == len(list(m.parameters()))
    assert max(errs.values()) < 8e-2, errs


@pytest.mark.parametrize("policy_logits", [False, True])
def test_gridnet_engine_behaviour_logp_matches_learner(cuda, policy_logits):
    """GridNet through the GPU actor engine: the captured policy step samples with the sparse
    active-cell logits (policy_logits=False) or the dense pixel-major ones (True, the emitted
    reference key); either way the behaviour log-prob of the first rollout equals what the
    learner scores for the same weights, obs, masks and actions (ratio 1 up to bf16)."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.gridnet import GridNetAgent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    s, T, E = 10, 8, 32

    def mk():
        return GridNetAgent((s, s, 27))

    torch.manual_seed(0)
    learner = Learner(mk(), LearnerHParams(), cuda)
    rt = GpuActorRuntime(mk, s, n_groups=1, envs_per_group=E, unroll=T, batch_slots=1,
                         device=cuda, n_threads=2, max_steps=50, policy_logits=policy_logits)
    rt.start(learner.flat)
    try:
        b, sl = rt.get_batch()
        torch.cuda.synchronize()
        batch = {k: v.clone() for k, v in b.items()}
        rt.release(sl)
    finally:
        rt.stop()
    m = learner.model
    obs = batch["obs"].reshape((T + 1) * E, -1)
    mask = batch["mask"][:T].reshape(T * E, s * s, 3)
    act = batch["action"][:T].reshape(T * E, s * s, 7)
    with torch.no_grad():
        lp, _, _ = m.evaluate(obs, mask, act, n_score=T * E)
    active = (mask != 0).any(-1).sum().item()
    assert active > 0
    torch.testing.assert_close(lp, batch["logp"][:T].reshape(-1), rtol=2e-2, atol=5e-2)
    if policy_logits:
        assert batch["policy_logits"].shape[-1] == s * s * 78
