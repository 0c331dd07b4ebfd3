"""Reference-compatible ``Agent.get_action`` / ``get_value`` on the GPU run the HIP kernels
(reference model.py:165-220 API): dense float one-hot obs are packed to bit planes, the
trunk is conv.hip/trunk.hip, the dense actor logits come from gemm.hip, and the masked
categoricals from masked_cell.hip. Checked against the same call on the CPU (PyTorch fp32
reference semantics) with bf16 tolerances; unsupported conv widths fail loudly."""
import pytest
import torch

from microbeast_amd.ops import cell_head
from microbeast_amd.ops.obs import bits_to_dense

pytestmark = pytest.mark.gpu


def _inputs(s, n, seed=0):
    from microbeast_amd import _native as N
    rt = N.runtime()
    env = rt.VecEnv(s, n, 400, seed, [0, 1, 2, 3])
    codes = torch.zeros(n, s * s, dtype=torch.int16)
    res = torch.zeros(n, dtype=torch.int32)
    rew, done = torch.zeros(n), torch.zeros(n, dtype=torch.uint8)
    env.reset(0, 0)
    g = torch.Generator().manual_seed(seed)
    for _ in range(20):
        a16 = torch.randint(0, 1 << 14, (n, s * s), generator=g, dtype=torch.int32).to(torch.int16)
        env.step_codes(a16.data_ptr(), codes.data_ptr(), res.data_ptr(), rew.data_ptr(), done.data_ptr())
    k = N.kernels()
    dev = torch.device("cuda", 0)
    obs = torch.empty(n, s * s, dtype=torch.int32, device=dev)
    mask = torch.empty(n, s * s, 3, dtype=torch.int32, device=dev)
    N.check(k.mbk_decode_obs_mask(codes.to(dev).data_ptr(), res.to(dev).data_ptr(), n, s, s,
                                  obs.data_ptr(), mask.data_ptr(), N.stream_ptr()), "decode")
    dense = bits_to_dense(obs, s, s)                      # (n, s, s, 27) float one-hot
    mask78 = cell_head.unpack_mask(mask).reshape(n, -1).to(torch.uint8)  # (n, 78 s s)
    return dense, mask78


def test_get_action_learning_matches_cpu(cuda):
    from microbeast_amd.models.agent import Agent
    s, n = 8, 24
    dense, mask78 = _inputs(s, n)
    torch.manual_seed(0)
    cpu = Agent((s, s, 27))
    torch.nn.init.normal_(cpu.actor.weight, std=0.05)
    gpu = Agent((s, s, 27))
    gpu.load_state_dict(cpu.state_dict())
    gpu = gpu.to(cuda)
    # actions sampled on the CPU under the mask, then scored by both
    with torch.no_grad():
        out_c, _ = cpu.get_action({"obs": dense.cpu().view(1, 1, n, s, s, 27),
                                   "action_mask": mask78.cpu().view(1, n, -1)})
    act = out_c["action"]
    inp = {"obs": dense, "action_mask": mask78, "action": act.to(cuda)}
    out_g, _ = gpu.get_action(inp, learning=True)
    out_r, _ = cpu.get_action({k: v.cpu() for k, v in inp.items()}, learning=True)
    torch.cuda.synchronize()
    torch.testing.assert_close(out_g["policy_logits"].cpu(), out_r["policy_logits"],
                               rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(out_g["baseline"].cpu(), out_r["baseline"], rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(out_g["logprobs"].cpu(), out_r["logprobs"], rtol=3e-2, atol=0.1)
    torch.testing.assert_close(out_g["entropy"].cpu(), out_r["entropy"], rtol=3e-2, atol=0.1)
    v = gpu.get_value({"obs": dense.view(1, 1, n, s, s, 27)})
    torch.testing.assert_close(v.view(-1).cpu(), out_r["baseline"].view(-1), rtol=3e-2, atol=3e-2)


def test_get_action_sampling_is_legal(cuda):
    from microbeast_amd.models.agent import Agent
    s, n = 8, 32
    dense, mask78 = _inputs(s, n, seed=3)
    torch.manual_seed(1)
    gpu = Agent((s, s, 27)).to(cuda)
    out, _ = gpu.get_action({"obs": dense.view(1, 1, n, s, s, 27),
                             "action_mask": mask78.view(1, n, -1)})
    torch.cuda.synchronize()
    a = out["action"].view(n, s * s, 7).cpu()
    m = mask78.view(n, s * s, 78).bool().cpu()
    for k in range(7):
        seg = m[..., cell_head.OFFS[k]:cell_head.OFFS[k + 1]]
        ok = seg.gather(-1, a[..., k:k + 1]).squeeze(-1) | ~seg.any(-1)
        assert bool(ok.all()), f"illegal component {k}"
    assert out["policy_logits"].shape == (n, 78 * s * s) and out["logprobs"].shape == (n,)


def test_unsupported_width_fails_loudly(cuda):
    from microbeast_amd.models.agent import Agent
    m = Agent((8, 8, 27), channels=(8, 16, 16)).to(cuda)
    with pytest.raises(RuntimeError, match="hip_kernels=False"):
        m.policy_value(torch.zeros(2, 64, dtype=torch.int32, device=cuda))
