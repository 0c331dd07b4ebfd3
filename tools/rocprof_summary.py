#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into a small markdown table.

usage: python tools/rocprof_summary.py <rocprof_out_dir> <out.md> [--drop-trace]
"""
import csv
import glob
import os
import sys


def busy_report(trace_csv, window_frac=0.5):
    """GPU busy fraction (union of kernel intervals) over the last ``window_frac`` of the
    trace span, i.e. the steady state after warm-up, plus the busiest kernels there."""
    iv = []
    for r in csv.DictReader(open(trace_csv)):
        try:
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"),
                       r.get("Kernel_Name", "?")))
        except (KeyError, ValueError):
            continue
    if not iv:
        return []
    iv.sort()
    t_end = max(x[1] for x in iv)
    t0 = iv[0][0] + int((t_end - iv[0][0]) * (1.0 - window_frac))
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in iv:
        if e <= t0:
            continue
        s = max(s, t0)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = t_end - t0
    out = [f"### steady-state window ({os.path.basename(trace_csv)}, last {window_frac:.0%} of span)\n",
           f"span {span / 1e6:.2f} ms, GPU busy (union of kernels) {busy / 1e6:.2f} ms "
           f"= {100.0 * busy / max(span, 1):.1f} %\n"]
    # per hardware queue (policy stream vs learner stream vs RCCL): union of its kernels
    for q in sorted({x[2] for x in iv}):
        qb, cs, ce = 0, None, None
        names = {}
        for s, e, qq, nm in iv:
            if qq != q or e <= t0:
                continue
            names[nm] = names.get(nm, 0) + e - max(s, t0)
            s = max(s, t0)
            if ce is None or s > ce:
                if ce is not None:
                    qb += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        if ce is not None:
            qb += ce - cs
        if qb > 0.01 * span:
            top = max(names, key=names.get).replace("(anonymous namespace)::", "")[:60]
            out.append(f"- queue {q}: busy {qb / 1e6:.2f} ms = {100.0 * qb / max(span, 1):.1f} % "
                       f"(largest kernel: `{top}`)")
    out.append("")
    return out


def seq_report(trace_csv, last_n):
    """the last ``last_n`` dispatches in order: kernel, grid, duration (one learner update's
    layer-by-layer timeline when the program ends with it)"""
    rows = []
    for r in csv.DictReader(open(trace_csv)):
        try:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?"),
                         "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))))
        except (KeyError, ValueError):
            continue
    rows.sort()
    rows = rows[-last_n:]
    out = [f"### last {len(rows)} dispatches ({os.path.basename(trace_csv)})\n", "| # | kernel | grid | us |",
           "|---|---|---|---|"]
    for i, (s, e, nm, g) in enumerate(rows):
        nm = nm.replace("(anonymous namespace)::", "")
        out.append(f"| {i} | `{nm[:70]}` | {g} | {(e - s) / 1e3:.1f} |")
    out.append("")
    return out


def main():
    d, out = sys.argv[1], sys.argv[2]
    seq = 0
    for a in sys.argv[3:]:
        if a.startswith("--seq="):
            seq = int(a.split("=", 1)[1])
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
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        lines.extend(busy_report(f))
        if seq:
            lines.extend(seq_report(f, seq))
    open(out, "w").write("\n".join(lines) + "\n")
    if "--drop-trace" in sys.argv:
        for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            if "kernel_stats" not in f:
                os.remove(f)
    print("\n".join(lines[:60]))


if __name__ == "__main__":
    main()
