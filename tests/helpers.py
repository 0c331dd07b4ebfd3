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


def engine_batches(dev, S, n, groups=2, envs=32, T=8, seed=0, learn=True):
    """``n`` real rollout batches (cloned) from the GPU actor engine on an S x S map; the
    learner updates between them (so later batches are off-policy by the measured lag)."""
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    def mk():
        return Agent((S, S, 27))

    torch.manual_seed(seed)
    learner = Learner(mk(), LearnerHParams(), dev)
    rt = GpuActorRuntime(mk, S, n_groups=groups, envs_per_group=envs, unroll=T, batch_slots=1,
                         device=dev, n_threads=2, seed=seed + 1)
    rt.start(learner.flat)
    out = []
    try:
        for _ in range(n):
            b, slots = rt.get_batch(timeout=120)
            out.append({k: v.clone() for k, v in b.items()})
            if learn:
                learner.learn(b)
            rt.release(slots)
            rt.publish(learner.flat, version=learner.n_updates)
        torch.cuda.synchronize()
    finally:
        rt.stop()
    return out
