#!/usr/bin/env python
"""Inference encoder forward per frame at acting batch sizes: the fused LDS trunk
(trunk_tail_kernel, the captured graph's) vs the learner's per-stage kernels (save=False),
vs the learner forward (save=True). HIP-event timed, obs bits from random codes.

    python tools/enc_fwd_ab.py [--n 8192,32768]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="8192,32768")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.encoder import HipEncoder, encoder_params

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = Agent((16, 16, 27)).to(dev)
    params = [p.detach() for p in encoder_params(m.network, 3)]
    enc = HipEncoder(16, 16, 27, (16, 32, 32), dev)
    for n in [int(x) for x in a.n.split(",")]:
        codes = torch.randint(0, 1 << 26, (n, 256), dtype=torch.int32, device=dev)
        res = {}
        for name, fused, save in (("fused_tail", True, False), ("per_stage", False, False),
                                  ("learner_fwd", False, True)):
            enc.fused_tail = fused
            enc.forward(codes, params, save=save)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(a.iters):
                enc.forward(codes, params, save=save, prepacked=not save)
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / a.iters
            res[name] = {"us": round(1e3 * ms, 1), "ns_per_frame": round(1e6 * ms / n, 2)}
        print(json.dumps({"n": n, **res}), flush=True)


if __name__ == "__main__":
    main()
