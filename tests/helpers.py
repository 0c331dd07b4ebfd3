import torch

from microbeast_amd.ops.cell_head import pack_mask


def full_mask(n, S):
    return pack_mask(torch.ones(n, S, 78, dtype=torch.bool))


def synthetic_batch(model, T, B, S, seed, reward_fn=None, obs=None):
    """On-policy time-major batch [T+1, B, ...] sampled from ``model`` (CPU)."""
    g = torch.Generator().manual_seed(seed)
    if obs is None:
        obs = torch.randint(0, 2**26, ((T + 1) * B, S), dtype=torch.int32, generator=g)
    mask = full_mask((T + 1) * B, S)
    a, lp, v = model.act(obs, mask, generator=g)
    reward = reward_fn(a).float() if reward_fn else torch.randn((T + 1) * B, generator=g)
    return {
        "obs": obs.view(T + 1, B, S),
        "mask": mask.view(T + 1, B, S, 3),
        "action": a.view(T + 1, B, S, 7),
        "logp": lp.view(T + 1, B),
        "reward": reward.view(T + 1, B),
        "done": torch.zeros(T + 1, B, dtype=torch.uint8),
    }
