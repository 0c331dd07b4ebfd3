"""O(T) advantage scans vs the reference's O(T^2) loops (libs/utils.py:104-163)."""
import torch

from microbeast_amd.ops.advantages import advantages, flatten_batch_and_advantages, td_deltas


def _ref_deltas(r, v, d, gamma):
    n, T1 = r.shape
    out = torch.zeros(n, T1)
    for t in range(T1 - 1):
        out[:, t] = r[:, t] + gamma * v[:, t + 1] * (1 - d[:, t]) - v[:, t]
    return out


def _ref_adv(r, v, d, gamma):
    n, T1 = r.shape
    out = torch.zeros(n, T1)
    for t in range(T1 - 1):
        disc, acc = 1.0, torch.zeros(n)
        for k in range(t, T1 - 1):
            acc = acc + disc * (r[:, k] + gamma * v[:, k + 1] * (1 - d[:, k]) - v[:, k])
            disc *= gamma
        out[:, t] = acc
    return out


def test_deltas_and_reference_advantages():
    g = torch.Generator().manual_seed(0)
    r, v = torch.randn(5, 17, generator=g), torch.randn(5, 17, generator=g)
    d = (torch.rand(5, 17, generator=g) < 0.15).float()
    torch.testing.assert_close(td_deltas(r, v, d, 0.99), _ref_deltas(r, v, d, 0.99))
    torch.testing.assert_close(advantages(r, v, d, 0.99, reference=True), _ref_adv(r, v, d, 0.99),
                               rtol=1e-5, atol=1e-5)


def test_gae_stops_at_episode_end():
    r = torch.tensor([[1.0, 1.0, 1.0, 0.0]])
    v = torch.zeros(1, 4)
    d = torch.tensor([[0.0, 1.0, 0.0, 0.0]])
    a = advantages(r, v, d, 0.5, lam=1.0)
    assert torch.allclose(a, torch.tensor([[1.5, 1.0, 1.0, 0.0]]))


def test_flatten_layout():
    b = {"obs": torch.zeros(3, 5, 4, 4, 27), "reward": torch.zeros(3, 5), "ep_step": torch.zeros(3, 5)}
    fb, fa = flatten_batch_and_advantages(b, torch.zeros(3, 5))
    assert fb["obs"].shape == (1, 15, 4, 4, 27) and fb["reward"].shape == (1, 15)
    assert fb["ep_step"].shape == (15,) and fa.shape == (15,)
