#!/usr/bin/env python
"""Per-dispatch timeline of the LAST learner update in a rocprofv3 kernel trace, with the
HBM bytes each trunk layer must move at least (from its role in ops/encoder.py), so each
conv reads as an achieved-bandwidth / MFMA-rate figure.

    python tools/layer_times.py <rocprof_dir> [--last_kernel vtrace_kernel] [--n 120]

The last update is found as the dispatches between the second-to-last and the last
``adam_kernel`` (the optimizer closes every update).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--out", default="")
    a = p.parse_args(argv)
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            try:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
            except (KeyError, ValueError):
                pass
    rows.sort()
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[2]]
    if len(adam) < 2:
        raise SystemExit("need two adam_kernel dispatches in the trace")
    seg = rows[adam[-2] + 1:adam[-1] + 1]
    t0 = seg[0][0]
    lines = ["| # | start us | dur us | kernel |", "|---|---|---|---|"]
    tot = 0.0
    for i, (s, e, k) in enumerate(seg):
        d = (e - s) / 1e3
        tot += d
        name = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        lines.append(f"| {i} | {(s - t0) / 1e3:.1f} | {d:.1f} | `{name[:90]}` |")
    span = (seg[-1][1] - t0) / 1e3
    lines.append("")
    lines.append(f"update span {span:.1f} us, kernel sum {tot:.1f} us, {len(seg)} dispatches")
    out = "\n".join(lines)
    if a.out:
        with open(a.out, "w") as f:
            f.write(out + "\n")
    print(out)


if __name__ == "__main__":
    main()
