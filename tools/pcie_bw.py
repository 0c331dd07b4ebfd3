#!/usr/bin/env python
"""Pinned host <-> HBM copy latency/bandwidth at the engine's per-step sizes, alone and
while another stream keeps the GPU busy with HBM-heavy kernels (the learner's situation).

    python tools/pcie_bw.py
"""
import json
import time

import torch


def timed(fn, iters=50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev, priority=-1)
    for mb in (0.5, 1, 2, 4, 8):
        n = int(mb * (1 << 20))
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        with torch.cuda.stream(s):
            h2d = timed(lambda: d.copy_(h, non_blocking=True))
            d2h = timed(lambda: h.copy_(d, non_blocking=True))
        # background HBM load on the default stream
        big = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        big2 = torch.empty_like(big)
        for _ in range(20):
            big2.copy_(big)
        with torch.cuda.stream(s):
            h2d_l = timed(lambda: d.copy_(h, non_blocking=True), 20)
            d2h_l = timed(lambda: h.copy_(d, non_blocking=True), 20)
        torch.cuda.synchronize()
        del big, big2
        print(json.dumps({"MiB": mb, "h2d_us": round(h2d * 1e6, 1), "d2h_us": round(d2h * 1e6, 1),
                          "h2d_GBs": round(n / h2d / 1e9, 1), "d2h_GBs": round(n / d2h / 1e9, 1),
                          "h2d_loaded_us": round(h2d_l * 1e6, 1),
                          "d2h_loaded_us": round(d2h_l * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
