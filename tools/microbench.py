#!/usr/bin/env python
"""Isolated GPU timings: policy step (captured graph replay) and learner update.

    python tools/microbench.py [--size 16] [--E 256,1024] [--learn_frames 32768]
Prints one JSON line per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=16)
    p.add_argument("--arch", default="impala_flat", help="impala_flat | gridnet | impala_deep")
    p.add_argument("--E", type=str, default="256,1024")
    p.add_argument("--learn_T", type=int, default=64)
    p.add_argument("--learn_B", type=str, default="512,1024")
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--policy_eager", action="store_true",
                   help="also run the policy step eagerly (no graph) so rocprof sees its kernels")
    p.add_argument("--fp8", action="store_true", help="policy step on the fp8 acting trunk")
    p.add_argument("--no_learner", action="store_true", help="policy step timings only")
    a = p.parse_args()
    import torch

    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.runtime.gpu_actors import GpuActorRuntime

    dev = torch.device("cuda", 0)
    s = a.size
    if a.arch == "gridnet":
        from microbeast_amd.models.gridnet import GridNetAgent
        mk = lambda: GridNetAgent((s, s, 27))  # noqa: E731
    elif a.arch == "impala_deep":
        mk = lambda: Agent((s, s, 27), channels=(16, 32, 32, 32))  # noqa: E731
    else:
        mk = lambda: Agent((s, s, 27))  # noqa: E731
    for E in [int(x) for x in a.E.split(",") if x]:
        rt = GpuActorRuntime(mk, s, 1, E, 8, 1, dev, n_threads=1, fp8_policy=a.fp8)
        # realistic inputs: run the env once to get observations / masks
        env = rt.engine.env  if hasattr(rt.engine, "env") else None  # noqa: F841
        g = rt.graph
        for _ in range(5):
            g.replay()
        if os.environ.get("MBK_MICRO_POLICY_ITERS"):
            a.iters = int(os.environ["MBK_MICRO_POLICY_ITERS"])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        print(json.dumps({"what": "policy_step_graph", "arch": a.arch, "E": E, "fp8": a.fp8,
                          "trunk8": os.environ.get("MBK_TRUNK8", "1"), "ms": round(dt * 1e3, 4),
                          "frames_per_s": round(E / dt, 1)}), flush=True)
        if a.policy_eager:
            for _ in range(a.iters):
                rt._policy_step(rt.io, rt.infer_model, rt.rng)
            torch.cuda.synchronize()
        del rt
    if a.no_learner:
        return
    torch.manual_seed(0)
    learner = Learner(mk(), LearnerHParams(), dev)
    from microbeast_amd.envs.synthetic import create_env

    T = a.learn_T
    for B in [int(x) for x in a.learn_B.split(",") if x]:
        env = create_env(s, B, 2000, seed=1)
        S = s * s
        obs = torch.zeros(T + 1, B, S, dtype=torch.int32)
        mask = torch.zeros(T + 1, B, S, 3, dtype=torch.int32)
        env.reset_compact(obs[0], mask[0])
        act = torch.zeros(T + 1, B, S, 7, dtype=torch.uint8)
        rew = torch.zeros(T + 1, B)
        done = torch.zeros(T + 1, B, dtype=torch.uint8)
        m = learner.model
        for t in range(T + 1):
            with torch.no_grad():
                at, _, _ = m.act(obs[t].to(dev), mask[t].to(dev),
                                 torch.tensor([1, t], dtype=torch.int64, device=dev))
            act[t] = at.cpu()
            if t < T:
                o2, m2, r2, d2 = env.step_compact(act[t])
                obs[t + 1], mask[t + 1], rew[t], done[t] = o2, m2, r2, d2
        batch = {"obs": obs.to(dev), "mask": mask.to(dev), "action": act.to(dev),
                 "logp": torch.zeros(T + 1, B, device=dev), "reward": rew.to(dev),
                 "done": done.to(dev)}
        active = int((mask.view(-1, 3) != 0).any(-1).sum())
        for variant in [""]:
            for _ in range(3):
                learner.learn(batch)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = max(3, a.iters // 5)
            for _ in range(n):
                learner.learn(batch)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            learner.learn(batch, sync_timing=True)
            print(json.dumps({"what": "learner_update", "variant": variant or "default",
                              "frames": T * B, "ms": round(dt * 1e3, 3),
                              "frames_per_s": round(T * B / dt, 1),
                              "active_cells_frac": round(active / ((T + 1) * B * S), 4),
                              "phases_s": learner.timing}), flush=True)


if __name__ == "__main__":
    main()
