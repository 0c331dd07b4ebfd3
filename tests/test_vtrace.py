"""V-trace + losses vs a straightforward NumPy double-loop oracle (Espeholt et al. 2018)."""
import numpy as np
import torch

from microbeast_amd.ops.vtrace import vtrace_torch


def _oracle(lpn, lpo, values, rewards, dones, gamma):
    T, B = lpn.shape
    ratio = np.exp(lpn - lpo)
    rho = np.minimum(1.0, ratio)
    c = np.minimum(1.0, ratio)
    disc = gamma * (1.0 - dones)
    v = values[:T]
    v_next = values[1:T + 1]
    vs = np.zeros((T, B))
    for b in range(B):
        for s in range(T):
            acc = 0.0
            prod = 1.0
            gpow = 1.0
            for t in range(s, T):
                delta = rho[t, b] * (rewards[t, b] + disc[t, b] * v_next[t, b] - v[t, b])
                acc += gpow * prod * delta
                prod *= c[t, b]
                gpow *= disc[t, b]
            vs[s, b] = v[s, b] + acc
    vs_next = np.concatenate([vs[1:], values[T:T + 1]], 0)
    adv = np.minimum(1.0, ratio) * (rewards + disc * vs_next - v)
    return vs, adv


def test_vtrace_matches_oracle():
    rng = np.random.default_rng(0)
    T, B = 9, 5
    lpn = rng.normal(-3, 0.3, (T, B))
    lpo = lpn + rng.normal(0, 0.3, (T, B))
    values = rng.normal(0, 1, (T + 1, B))
    rewards = rng.normal(0, 1, (T, B))
    dones = (rng.random((T, B)) < 0.2).astype(np.float64)
    vs, adv = _oracle(lpn, lpo, values, rewards, dones, 0.99)
    out = vtrace_torch(torch.tensor(lpn, dtype=torch.float32), torch.tensor(lpo, dtype=torch.float32),
                       torch.tensor(values, dtype=torch.float32), torch.tensor(rewards, dtype=torch.float32),
                       torch.tensor(dones.astype(bool)), None, gamma=0.99)
    np.testing.assert_allclose(out.vs.numpy(), vs, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(out.adv.numpy(), adv, rtol=1e-4, atol=1e-4)


def test_gradients_equal_autograd_of_losses():
    torch.manual_seed(0)
    T, B = 6, 4
    lpn = (torch.randn(T, B) - 3).requires_grad_(True)
    lpo = lpn.detach() + 0.1 * torch.randn(T, B)
    val = torch.randn(T + 1, B, requires_grad=True)
    rew = torch.randn(T, B)
    done = torch.rand(T, B) < 0.2
    ent = torch.rand(T, B, requires_grad=True)
    out = vtrace_torch(lpn, lpo, val, rew, done, ent, baseline_cost=0.5, entropy_cost=0.01)
    vs, adv = out.vs.detach(), out.adv.detach()
    pg = -(lpn * adv).mean()                      # correct sign (reference D4 had +)
    vl = 0.5 * ((vs - val[:T]) ** 2).mean()        # reference libs/utils.py:323
    el = ent.mean()
    total = pg + vl - 0.01 * el
    total.backward()
    torch.testing.assert_close(lpn.grad, out.g_logp)
    torch.testing.assert_close(val.grad, out.g_value)
    torch.testing.assert_close(ent.grad, torch.full_like(ent, out.g_ent))
    torch.testing.assert_close(out.losses[3], total.detach(), rtol=1e-5, atol=1e-6)
