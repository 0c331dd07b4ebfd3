"""Model architecture parity with the reference Agent (names, shapes, counts, API)."""
import torch

from microbeast_amd.models.agent import Agent, num_params
from microbeast_amd.models.gridnet import GridNetAgent


def test_param_counts_match_reference():
    # SURVEY §7.6 (probed on the reference model.py)
    expected = {4: 430_497, 8: 1_392_705, 10: 2_138_937, 16: 5_266_113, 24: 11_721_793}
    for s, n in expected.items():
        assert num_params(Agent((s, s, 27))) == n, s


def test_state_dict_keys_follow_reference_names():
    sd = Agent((16, 16, 27)).state_dict()
    assert sd["network.0.conv.weight"].shape == (16, 27, 3, 3)
    assert sd["network.1.conv.weight"].shape == (32, 16, 3, 3)
    assert sd["network.2.res_block1.conv1.weight"].shape == (32, 32, 3, 3)
    assert sd["network.5.weight"].shape == (256, 128)
    assert sd["actor.weight"].shape == (19968, 256)
    assert sd["critic.weight"].shape == (1, 256)
    assert torch.count_nonzero(sd["actor.weight"]) == 0  # orthogonal gain 0 (model.py:136)


def test_reference_get_action_api():
    torch.manual_seed(0)
    s, n = 8, 6
    m = Agent((s, s, 27), [6, 4, 4, 4, 4, 7, 49] * (s * s), s * s, "cpu")
    obs = torch.zeros(1, 1, n, s, s, 27)
    obs[..., 0] = 1
    mask = (torch.rand(1, n, 78 * s * s) < 0.3).to(torch.uint8)
    out, state = m.get_action({"obs": obs, "action_mask": mask})
    assert state == ()
    assert out["action"].shape == (n, 7 * s * s)
    assert out["policy_logits"].shape == (n, 78 * s * s)
    assert out["logprobs"].shape == (n,) and out["baseline"].shape == (1, n)
    lo, _ = m.get_action({"obs": obs.view(n, s, s, 27), "action_mask": mask.view(n, -1),
                          "action": out["action"]}, learning=True)
    torch.testing.assert_close(lo["logprobs"], out["logprobs"])
    assert lo["entropy"].shape == (n,)


def test_act_evaluate_consistent_cpu():
    torch.manual_seed(0)
    m = Agent((4, 4, 27))
    obs = torch.randint(0, 2**26, (5, 16), dtype=torch.int32)
    mask = torch.randint(-2**31, 2**31 - 1, (5, 16, 3), dtype=torch.int32)
    a, lp, v = m.act(obs, mask, generator=torch.Generator().manual_seed(1))
    lp2, ent, v2 = m.evaluate(obs, mask, a)
    torch.testing.assert_close(lp, lp2.detach())
    torch.testing.assert_close(v, v2.detach())


def test_gridnet_shapes():
    m = GridNetAgent((16, 16, 27), compute_dtype=torch.float32)
    obs = torch.randint(0, 2**26, (3, 256), dtype=torch.int32)
    logits, v = m.policy_value(obs)
    assert logits.shape == (3, 256 * 78) and v.shape == (3,)
    m10 = GridNetAgent((10, 10, 27), compute_dtype=torch.float32)
    logits, v = m10.policy_value(torch.randint(0, 2**26, (2, 100), dtype=torch.int32))
    assert logits.shape == (2, 100 * 78)
