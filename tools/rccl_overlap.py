#!/usr/bin/env python
"""RCCL all-reduce kernels of the last learner update in a rocprofv3 kernel trace, and the
learner kernels they overlap (bench.py with MBK_FORCE_PG=1: a real RCCL group at world 1).

    python tools/rccl_overlap.py <rocprof_dir>
"""
from __future__ import annotations

import csv
import glob
import os
import sys


def short(k: str) -> str:
    return k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]


def main(d: str) -> None:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[2]]
    if len(adam) < 2:
        raise SystemExit("need two adam_kernel dispatches")
    s0 = rows[adam[-2]][1]
    seg = [r for r in rows if s0 < r[0] <= rows[adam[-1]][1]]
    rccl = [r for r in seg if "nccl" in r[2].lower() or "rccl" in r[2].lower()]
    other = [r for r in seg if r not in rccl]
    print(f"last update: {len(seg)} kernels, {len(rccl)} RCCL")
    for s, e, k in rccl:
        ov = sorted({short(k2) for s2, e2, k2 in other if s2 < e and e2 > s})
        print(f"  {(s - s0) / 1e3:9.1f} us +{(e - s) / 1e3:7.1f} us  {short(k)}")
        print(f"      overlaps: {', '.join(ov) if ov else '(nothing)'}")


if __name__ == "__main__":
    main(sys.argv[1])
