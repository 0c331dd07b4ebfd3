#!/usr/bin/env python
"""Per-queue launch-gap analysis of a rocprofv3 kernel trace.

For every hardware queue: the kernels in start order, the idle gap before each one
(start minus the previous kernel's end on that queue), and per kernel name the median
duration and median preceding gap. Answers "how much of a captured graph's wall time is
kernel work and how much is dispatch/barrier overhead".

usage: python tools/trace_gaps.py <kernel_trace.csv | rocprof_out_dir> [--skip_frac 0.3]
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def load(path):
    if os.path.isdir(path):
        found = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))
        if not found:
            raise SystemExit(f"no kernel_trace.csv under {path}")
        path = found[0]
    rows = []
    for r in csv.DictReader(open(path)):
        try:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r.get("Queue_Id", "0"), r.get("Kernel_Name", "?")))
        except (KeyError, ValueError):
            continue
    rows.sort()
    return rows


def short(name, n=70):
    name = name.replace("(anonymous namespace)::", "")
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    path = sys.argv[1]
    skip = float(sys.argv[sys.argv.index("--skip_frac") + 1]) if "--skip_frac" in sys.argv else 0.3
    rows = load(path)
    if not rows:
        return
    t_first, t_last = rows[0][0], max(r[1] for r in rows)
    t0 = t_first + int((t_last - t_first) * skip)
    by_q = defaultdict(list)
    for r in rows:
        if r[0] >= t0:
            by_q[r[2]].append(r)
    for q, ks in sorted(by_q.items(), key=lambda kv: -len(kv[1])):
        span = ks[-1][1] - ks[0][0]
        busy = sum(e - s for s, e, _, _ in ks)
        print(f"queue {q}: {len(ks)} kernels, span {span / 1e6:.2f} ms, "
              f"kernel time {busy / 1e6:.2f} ms ({100.0 * busy / max(span, 1):.1f} %)")
        dur, gap = defaultdict(list), defaultdict(list)
        prev_end = None
        for s, e, _, name in ks:
            dur[name].append(e - s)
            if prev_end is not None:
                gap[name].append(max(0, s - prev_end))
            prev_end = max(prev_end or 0, e)
        print(f"  {'kernel':70s} {'calls':>6s} {'med us':>8s} {'med gap us':>10s}")
        for name in sorted(dur, key=lambda n: -sum(dur[n]))[:20]:
            g = statistics.median(gap[name]) / 1e3 if gap[name] else 0.0
            print(f"  {short(name):70s} {len(dur[name]):6d} "
                  f"{statistics.median(dur[name]) / 1e3:8.2f} {g:10.2f}")


if __name__ == "__main__":
    main()
