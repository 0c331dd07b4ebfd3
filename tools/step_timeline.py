#!/usr/bin/env python
"""Timeline of the GPU actor engine's policy steps from a rocprofv3 trace.

Needs ``--kernel-trace --memory-copy-trace`` output (csv). For each policy step (anchored on
the decode kernel) it finds the host->device copy that precedes it and the device->host copy
that follows it, and reports medians (us) of: H2D duration, H2D end -> decode start, the
kernel span decode -> last policy kernel, -> D2H start, D2H duration, and the whole phase.

usage: python tools/step_timeline.py <rocprof_out_dir> [--skip_frac 0.5]
"""
from __future__ import annotations

import csv
import glob
import os
import statistics
import sys


def _load(d, pat):
    f = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    skip = float(sys.argv[sys.argv.index("--skip_frac") + 1]) if "--skip_frac" in sys.argv else 0.5
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
          for r in _load(d, "*kernel_trace.csv")]
    cs = []
    for r in _load(d, "*memory_copy_trace.csv"):
        direction = r.get("Direction", "")
        cs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), direction,
                   int(r.get("Size", 0) or 0)))
    ks.sort()
    cs.sort()
    if not ks:
        raise SystemExit("no kernel trace")
    t0 = ks[0][0] + skip * (ks[-1][1] - ks[0][0])
    dec = [k for k in ks if "decode_obs_mask" in k[2] and k[0] >= t0]
    h2d = [c for c in cs if "HOST_TO_DEVICE" in c[2].upper() and c[3] >= 1 << 20]
    d2h = [c for c in cs if "DEVICE_TO_HOST" in c[2].upper() and c[3] >= 1 << 20]
    pol_names = ("decode_obs_mask", "conv_fwd_kernel<32, 16, true", "trunk_tail", "fc_fwd",
                 "head_units", "head_fwd", "row_sum", "pack_env_actions", "multi_copy")
    rows = {k: [] for k in ("h2d_us", "h2d_to_decode_us", "kernels_us", "to_d2h_us", "d2h_us",
                            "phase_us")}
    import bisect
    h2d_end = [c[1] for c in h2d]
    d2h_start = [c[0] for c in d2h]
    for s, e, _ in dec:
        i = bisect.bisect_right(h2d_end, s) - 1
        if i < 0:
            continue
        hs, he = h2d[i][0], h2d[i][1]
        # last policy kernel of this step: policy kernels after decode, before the next decode
        j = bisect.bisect_left(d2h_start, s)
        if j >= len(d2h):
            continue
        ds, de = d2h[j][0], d2h[j][1]
        last = max((k[1] for k in ks if s <= k[0] < ds and any(p in k[2] for p in pol_names)),
                   default=e)
        rows["h2d_us"].append((he - hs) / 1e3)
        rows["h2d_to_decode_us"].append((s - he) / 1e3)
        rows["kernels_us"].append((last - s) / 1e3)
        rows["to_d2h_us"].append((ds - last) / 1e3)
        rows["d2h_us"].append((de - ds) / 1e3)
        rows["phase_us"].append((de - hs) / 1e3)
    print(f"steps analysed: {len(rows['phase_us'])} (H2D copies >= 1 MiB: {len(h2d)}, "
          f"D2H: {len(d2h)})")
    for k, v in rows.items():
        if v:
            q = statistics.quantiles(v, n=10) if len(v) > 10 else [min(v)] * 9
            print(f"  {k:18s} median {statistics.median(v):9.1f}   p10 {q[0]:9.1f}   "
                  f"p90 {q[-1]:9.1f}")


if __name__ == "__main__":
    main()
