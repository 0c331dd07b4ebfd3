"""How sensitive is the stage-2 block-1 conv0 weight gradient (network.2.res_block1.conv0,
2x2 maps) to rounding-level sign flips of its relu gate? (CPU, fp32.)

On a realistic 16x16 batch (real simulator games, uniform-legal actions) the fp32 learner's
stage-2 operands are captured: y0 (block input), u1 (conv0 output = the relu gate of du), g
(stage output gradient). The gradient is then recomputed with u1 perturbed by Gaussian noise of
bf16-rounding size (relative 2^-9 of |u1|, plus the absolute error a bf16 conv of bf16 inputs
makes: --abs) for many draws: each draw flips a handful of near-zero gates, and the spread of
the resulting dW errors is the floor ANY bf16 implementation faces on this layer. The GPU
probe (tools/dbg/parity_operand_swap.py) measured: HIP u1 error 0.4 % (torch-bf16 0.96 %),
171 flips (torch-bf16 204), but the HIP flips gate 1 % of |du| (torch-bf16 0.13 %) and give a
10 % dW error (torch-bf16 0.8 %).

    python tools/dbg/relu_flip_sensitivity.py [--draws 200]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def real_obs(E: int, steps: int, seed: int) -> torch.Tensor:
    from calibrate_env import uniform_legal

    from microbeast_amd import _native as N
    rt = N.runtime()
    S = 256
    env = rt.VecEnv(16, E, 2000, seed, [0, 0, 0, 1, 2, 3])
    obs = torch.zeros(E, S, dtype=torch.int32)
    mask = torch.zeros(E, S, 3, dtype=torch.int32)
    env.reset(obs.data_ptr(), mask.data_ptr())
    rew, done = torch.zeros(E), torch.zeros(E, dtype=torch.uint8)
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(steps):
        a = torch.from_numpy(uniform_legal(mask.numpy(), rng))
        env.step(a.data_ptr(), obs.data_ptr(), mask.data_ptr(), rew.data_ptr(), done.data_ptr())
        out.append(obs.clone())
    return torch.stack(out)  # [T, E, S]


def capture(args):
    from helpers import synthetic_batch

    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    torch.manual_seed(7)
    m = Agent((16, 16, 27), hip_kernels=False, compute_dtype=torch.float32)
    with torch.no_grad():
        m.actor.weight.normal_(0, 0.02)
        m.actor.bias.normal_(0, 0.02)
    T, B = args.T, args.envs
    obs = real_obs(B, T + 1 + 40, seed=args.seed)[40:].reshape(-1, 256)
    batch = synthetic_batch(m, T, B, 256, seed=args.seed, obs=obs)
    st2 = m.network[2]
    cap = {}
    st2.res_block1.register_forward_pre_hook(lambda mod, inp: cap.__setitem__("y0", inp[0].detach()))
    st2.res_block1.conv0.register_forward_hook(lambda mod, i, o: cap.__setitem__("u1", o.detach()))

    def yhook(mod, i, o):
        o.register_hook(lambda g: cap.__setitem__("g", g.detach()))
    st2.register_forward_hook(yhook)
    w1 = st2.res_block1.conv1.weight.detach().double().clone()
    L = Learner(m, LearnerHParams(), torch.device("cpu"))
    L.learn(batch)
    return {k: v.double() for k, v in cap.items()}, w1


def dw(y0, u1, g, w1):
    du1 = torch.nn.grad.conv2d_input(u1.shape, w1, g, padding=1) * (u1 > 0)
    return torch.nn.grad.conv2d_weight(F.relu(y0), (32, 32, 3, 3), du1, padding=1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=64)
    p.add_argument("--T", type=int, default=8)
    p.add_argument("--seed", type=int, default=16)
    p.add_argument("--draws", type=int, default=200)
    p.add_argument("--abs", type=float, default=1.5e-4,
                   help="absolute u1 error std of a bf16 conv (GPU probe: 1.3-2.0e-4 per channel)")
    args = p.parse_args()
    cap, w1 = capture(args)
    y0, u1, g = cap["y0"], cap["u1"], cap["g"]
    ref = dw(y0, u1, g, w1)
    rel = lambda a, c: float((a - c).norm() / c.norm())  # noqa: E731
    gen = torch.Generator().manual_seed(0)
    out = []
    du = torch.nn.grad.conv2d_input(u1.shape, w1, g, padding=1)
    for _ in range(args.draws):
        noise = (torch.randn(u1.shape, generator=gen, dtype=torch.float64)
                 * (args.abs + u1.abs() * 2.0 ** -9))
        up = u1 + noise
        flip = (up > 0) != (u1 > 0)
        out.append((rel(dw(y0, up, g, w1), ref), int(flip.sum()),
                    float(du[flip].abs().sum() / du.abs().sum())))
    r = np.array([o[0] for o in out])
    nf = np.array([o[1] for o in out])
    share = np.array([o[2] for o in out])
    print(f"{len(r)} draws at bf16-level u1 noise: flips median {np.median(nf):.0f}; dW rel error "
          f"median {np.median(r):.4f}, p90 {np.percentile(r, 90):.4f}, max {r.max():.4f}")
    print(f"corr(dW error, |du| share gated by the flips) = {np.corrcoef(r, share)[0, 1]:.3f}; "
          f"share median {np.median(share):.4f} max {share.max():.4f}")
    return r


if __name__ == "__main__":
    main()
