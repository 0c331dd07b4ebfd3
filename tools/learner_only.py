#!/usr/bin/env python
"""Learner updates only (synthetic engine-shaped batch), for kernel traces / counter passes
without acting kernels in the trace.

    python tools/learner_only.py --batch 8192 --T 64 --steps 2
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="impala_flat")
    ap.add_argument("--size", type=int, default=16)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--active", type=float, default=0.007,
                    help="fraction of (frame, cell) pairs with a legal action: 0.007 ~ the random-"
                         "init policy's early game, 0.025 ~ a settled training run (6.5 / 256)")
    ap.add_argument("--no_abits", action="store_true",
                    help="no active-cell bitmap rows in the batch (the head counts from masks)")
    ap.add_argument("--set", action="append", default=[],
                    help="enc.<attr>=<int> / head.<attr>=<int>: set a variant attribute of the "
                         "HIP encoder / sparse head before the first update (A/B in one process); "
                         "native.<setter>=<int>: call a kernel-library setter")
    ap.add_argument("--lib", default=None, help="variant library dir (tools/variant.py)")
    ap.add_argument("--bwd_occ", type=int, default=0,
                    help="backward workgroups per CU (the GPU actor runtime's cap is 1; 0: none)")
    ap.add_argument("--fwd_occ", type=int, default=0, help="forward workgroups per CU (as --bwd_occ)")
    a = ap.parse_args()
    import torch

    from tools.variant import use_lib
    use_lib(a.lib)
    if a.bwd_occ or a.fwd_occ:
        from microbeast_amd import _native as N
        N.check(N.kernels().mbk_set_learner_occupancy(a.fwd_occ, a.bwd_occ), "set_learner_occupancy")

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
    # sparse legal-action masks with --active of the cells live, like the engine's rollouts
    mask = torch.zeros(T + 1, B, S, 3, dtype=torch.int32, device=dev)
    act = torch.rand(T + 1, B, S, device=dev, generator=g) < a.active
    mask[..., 0] = torch.where(act, torch.randint(1, 2 ** 31 - 1, (T + 1, B, S), device=dev,
                                                  generator=g, dtype=torch.int32), 0)
    batch = {
        "obs": torch.randint(0, 2 ** 26, (T + 1, B, S), dtype=torch.int32, device=dev, generator=g),
        "mask": mask,
        "action": torch.zeros(T + 1, B, S, 7, dtype=torch.uint8, device=dev),
        "logp": -torch.rand(T + 1, B, device=dev, generator=g),
        "reward": torch.randn(T + 1, B, device=dev, generator=g),
        "done": torch.zeros(T + 1, B, dtype=torch.uint8, device=dev),
    }
    if not a.no_abits and S % 32 == 0:  # what the fused acting step writes with the rollout
        live = (mask != 0).any(-1).view(T + 1, B, S // 32, 32).to(torch.int64)
        w = (live << torch.arange(32, device=dev)).sum(-1)
        batch["abits"] = torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)
    learner.learn(batch)
    for kv in a.set:
        k, v = kv.split("=")
        obj, attr = k.split(".")
        if obj == "native":  # a kernel-library setter: native.mbk_x_set=<int>
            from microbeast_amd import _native as N
            getattr(N.kernels(), attr)(*[int(x) for x in v.split(":")])  # a:b -> two ints
            continue
        m = learner.model
        tgt = m._hip_enc if obj == "enc" else m._head(dev)
        assert hasattr(tgt, attr), kv
        setattr(tgt, attr, type(getattr(tgt, attr))(int(v)))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        learner.learn(batch)
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / a.steps * 1e3:.3f} ms per update "
          f"({(T * B) / 1e3:.0f}K frames)", flush=True)


if __name__ == "__main__":
    main()
