#!/usr/bin/env python
"""How long the acting kernels take under each learner kernel (rocprofv3 --kernel-trace CSV of
bench.py): the acting launches share the GPU with the learner's persistent kernels, whose
workgroups hold their CU slots until the kernel ends, so an acting kernel's duration depends on
what the learner runs beside it.

    python tools/acting_under.py <rocprof_out_dir> [window_frac=0.5] > out.md

For every act_trunk_w / head_act dispatch in the steady-state window (last ``window_frac`` of
the span), the learner kernel overlapping it longest (or none); per (acting kernel, learner
kernel): count, mean acting duration, and the learner kernel's launch resources (grid,
workgroup, LDS, VGPRs, as far as the trace reports them).
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict

ACT = ("act_trunk_w_kernel", "head_act_kernel")


def short(k: str) -> str:
    return k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]


def main(d: str, frac: float = 0.5) -> None:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(r)
    if not rows:
        raise SystemExit("no kernel_trace.csv under " + d)
    res_cols = [c for c in ("Grid_Size_X", "Grid_Size", "Workgroup_Size_X", "Workgroup_Size",
                            "Group_Segment_Size", "LDS_Block_Size", "Arch_VGPR_Count",
                            "Accum_VGPR_Count", "VGPR_Count", "SGPR_Count") if c in rows[0]]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r)
          for r in rows]
    iv.sort(key=lambda t: t[0])
    t_end = max(e for _, e, _, _ in iv)
    t_lo = t_end - frac * (t_end - iv[0][0])
    act = [t for t in iv if t[0] >= t_lo and t[2].startswith(ACT)]
    lrn = [t for t in iv if t[0] >= t_lo - 50e6 and not t[2].startswith(ACT)
           and not t[2].startswith("__amd")]
    res = {}
    for s, e, k, r in lrn:
        res.setdefault(k, {c: r[c] for c in res_cols})
    # sweep: learner kernels sorted by start; for each acting kernel scan the candidates
    stats = defaultdict(lambda: [0, 0.0])
    j0 = 0
    for s, e, k, _ in act:
        while j0 < len(lrn) and lrn[j0][1] < s - 100e6:
            j0 += 1
        best, bo = "(no learner kernel)", 0
        for ls, le, lk, _ in lrn[j0:]:
            if ls > e:
                break
            o = min(e, le) - max(s, ls)
            if o > bo:
                best, bo = lk, o
        st = stats[(k.split("_kernel")[0], best)]
        st[0] += 1
        st[1] += (e - s) / 1e3
    print(f"acting dispatches in the window: {len(act)}\n")
    print("| acting | longest-overlapping learner kernel | n | mean us | " +
          " | ".join(res_cols) + " |")
    print("|---|---|---|---|" + "---|" * len(res_cols))
    for (ak, lk), (n, tot) in sorted(stats.items(), key=lambda kv: (kv[0][0], -kv[1][1])):
        rr = res.get(lk, {})
        print(f"| {ak} | `{lk}` | {n} | {tot / n:.1f} | " +
              " | ".join(str(rr.get(c, "")) for c in res_cols) + " |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.5)
