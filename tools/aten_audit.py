#!/usr/bin/env python
"""Which Python lines still launch ATen / vendor-BLAS GPU kernels in a learner update?

Runs a few learner updates of ``--arch`` on synthetic engine-shaped batches under
torch.profiler (ROCm kineto) and prints, for every GPU kernel whose name is ATen
(``at::native``) or hipBLASLt (``Cijk``), the aten op that launched it and the innermost
frames of its Python stack. The goal state is an empty report.

    python tools/aten_audit.py --arch impala_flat --size 16 --batch 2048
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="impala_flat")
    ap.add_argument("--size", type=int, default=16)
    ap.add_argument("--batch", type=int, default=1024, help="envs per update (B)")
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from microbeast_amd.config import parse_flags
    from microbeast_amd.learner import Learner, LearnerHParams
    from microbeast_amd.models.factory import make_model

    dev = torch.device("cuda", 0)
    flags = parse_flags(["--device", "cuda", "--arch", a.arch, "--env_size", str(a.size),
                         "--quiet"], interactive=False)
    torch.manual_seed(0)
    learner = Learner(make_model(flags, dev), LearnerHParams(), dev)
    S, T, B = a.size * a.size, a.T, a.batch
    g = torch.Generator(device=dev).manual_seed(1)
    batch = {
        "obs": torch.randint(0, 2 ** 26, (T + 1, B, S), dtype=torch.int32, device=dev, generator=g),
        "mask": torch.randint(0, 2 ** 31 - 1, (T + 1, B, S, 3), dtype=torch.int32, device=dev,
                              generator=g),
        "action": torch.randint(0, 4, (T + 1, B, S, 7), dtype=torch.uint8, device=dev, generator=g),
        "logp": -torch.rand(T + 1, B, device=dev, generator=g) * 50,
        "reward": torch.randn(T + 1, B, device=dev, generator=g),
        "done": torch.zeros(T + 1, B, dtype=torch.uint8, device=dev),
    }
    batch["mask"][..., 2] &= (1 << 14) - 1
    learner.learn(batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(a.steps):
            learner.learn(batch)
        torch.cuda.synchronize()
    events = prof.events()
    report = defaultdict(lambda: [0, 0.0])
    n_kern = 0
    for e in events:
        for k in getattr(e, "kernels", None) or []:
            n_kern += 1
            if "at::native" not in k.name and "Cijk" not in k.name:
                continue
            top = e
            while top.cpu_parent is not None and top.cpu_parent.name.startswith("aten::"):
                top = top.cpu_parent
            frames = []
            for src in (e, top):
                frames = [f for f in (src.stack or []) if "microbeast_amd" in f or "tools/" in f]
                if frames:
                    break
            key = (k.name[:90], top.name, " <- ".join(frames[:3]))
            report[key][0] += 1
            report[key][1] += k.duration
    print(f"{a.arch} {a.size}x{a.size} B={B} T={T}: {n_kern} GPU kernels in {a.steps} updates")
    if not report:
        print("no ATen / hipBLASLt kernels")
    for (kern, op, stack), (cnt, us) in sorted(report.items(), key=lambda kv: -kv[1][1]):
        print(f"{cnt:5d} calls {us / max(1, a.steps):9.1f} us/update  {op:28s} {kern}\n"
              f"        {stack}")


if __name__ == "__main__":
    main()
