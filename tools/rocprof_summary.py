#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into a small markdown table.

usage: python tools/rocprof_summary.py <rocprof_out_dir> <out.md> [--drop-trace]
"""
import csv
import glob
import os
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    stats = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True))
    lines = []
    for f in stats:
        rows = list(csv.DictReader(open(f)))
        tot = sum(float(r.get("TotalDurationNs", 0) or 0) for r in rows)
        lines.append(f"### {os.path.relpath(f, d)}\n")
        lines.append(f"total kernel time: {tot / 1e6:.3f} ms over {sum(int(r.get('Calls', 0) or 0) for r in rows)} calls\n")
        lines.append("| kernel | calls | total ms | avg us | % |")
        lines.append("|---|---|---|---|---|")
        rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0) or 0))
        for r in rows[:40]:
            name = r.get("Name", "?")
            if len(name) > 110:
                name = name[:107] + "..."
            t = float(r.get("TotalDurationNs", 0) or 0)
            c = int(r.get("Calls", 0) or 0)
            lines.append(f"| `{name}` | {c} | {t / 1e6:.3f} | {t / max(c, 1) / 1e3:.2f} | {100 * t / max(tot, 1):.1f} |")
        lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    if "--drop-trace" in sys.argv:
        for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            if "kernel_stats" not in f:
                os.remove(f)
    print("\n".join(lines[:60]))


if __name__ == "__main__":
    main()
