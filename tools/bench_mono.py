#!/usr/bin/env python
"""BASELINE config 2 shape: N CPU actor PROCESSES -> 1 MI355X learner.

Unlike ``bench.py`` (native env threads + on-GPU policy graph, the headline path), this
measures the reference-shaped runtime a gym-microRTS (JVM) user runs: spawned actor
processes stepping their own envs, a dynamic-batching GPU policy server in the learner
process (runtime/inference.py), shared-memory rollout slots uploaded by pinned DMA one
batch ahead of the learner (runtime/staging.py), HIP learner. Synthetic env, random-init
weights.

    python tools/bench_mono.py --actors 64 --envs 6 --size 10 --arch gridnet --steps 10
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
    p.add_argument("--actors", type=int, default=64)
    p.add_argument("--envs", type=int, default=6)
    p.add_argument("--size", type=int, default=10)
    p.add_argument("--arch", type=str, default="gridnet")
    p.add_argument("--unroll", type=int, default=64)
    p.add_argument("--batch", type=int, default=8, help="rollout slots per update")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--wait_ms", type=float, default=2.0)
    a = p.parse_args()
    import torch

    from microbeast_amd.config import parse_flags
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.factory import make_model
    from microbeast_amd.runtime.mono import MonoRuntime

    flags = parse_flags(["--runtime", "mono", "--device", "cuda", "--arch", a.arch,
                         "--env_size", str(a.size), "--n_actors", str(a.actors),
                         "--n_envs", str(a.envs), "--unroll_length", str(a.unroll),
                         "--batch_size", str(a.batch), "--inference_wait_ms", str(a.wait_ms),
                         "--quiet"], interactive=False)
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    learner = Learner(make_model(flags, dev), LearnerHParams(), dev)
    rt = MonoRuntime(flags, learner.flat.numel, device=dev,
                     make_model=lambda: make_model(flags, "cpu"))
    rt.publish(learner.flat.data)
    rt.start()
    rt.enable_prefetch(dev)

    def step():
        batch, _ = rt.get_batch(300.0)
        losses = learner.learn(batch)
        rt.publish(learner.flat.data)
        return losses

    try:
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        s0 = dict(rt.server.stats())
        t0 = time.perf_counter()
        for _ in range(a.steps):
            losses = step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        s1 = rt.server.stats()
    finally:
        rt.stop()
    frames = a.steps * a.batch * a.envs * a.unroll
    nb = s1["batches"] - s0["batches"]
    print(json.dumps({
        "metric": f"env frames/sec, {a.actors} CPU actor processes -> 1 MI355X learner",
        "value": round(frames / el, 1), "unit": "frames/s", "ms_per_update": round(1e3 * el / a.steps, 2),
        "config": {"arch": a.arch, "map": f"{a.size}x{a.size}", "actors": a.actors,
                   "envs_per_actor": a.envs, "unroll": a.unroll, "slots_per_update": a.batch,
                   "cpus": len(os.sched_getaffinity(0))},
        "server": {"batches_per_s": round(nb / el, 1),
                   "mean_actors_per_batch": round((s1["requests"] - s0["requests"]) / max(1, nb), 2)},
        "last_losses": [float(x) for x in losses.tolist()[:4]],
        "data": "synthetic env, random-init weights"}), flush=True)


if __name__ == "__main__":
    main()
