#!/usr/bin/env python
"""Kernel sequence of the last eager policy step in a rocprofv3 kernel trace of
``tools/microbench.py --policy_eager --no_learner`` (a step starts at its decode kernel).

    python tools/policy_kernels.py <rocprof_dir>
"""
from __future__ import annotations

import csv
import glob
import os
import sys


def main(d: str) -> None:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "decode_obs_mask" in r[2]]
    if len(starts) < 2:
        raise SystemExit("need two policy steps in the trace")
    seg = rows[starts[-2]:starts[-1]]
    t0 = seg[0][0]
    for s, e, k in seg:
        name = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:7.1f} us  {name[:80]}")
    print(f"{len(seg)} kernels, span {(seg[-1][1] - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
