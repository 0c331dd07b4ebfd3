#!/usr/bin/env python
"""Policy / learner overlap analysis of a bench.py kernel trace (rocprofv3 --kernel-trace CSV).

usage: python tools/timeline.py <rocprof_out_dir> [window_frac]

Splits the steady-state window (last ``window_frac`` of the span) by hardware queue: the
policy queue is the one running ``trunk_tail`` / ``act_trunk`` kernels, everything else with kernels is
"learner". A policy step starts at its ``decode_obs_mask`` (graph step) or ``act_trunk`` (fused step)
kernel. Reports per-step stream
time inside vs outside learner activity, per-queue busy and idle time, and the union.
"""
import csv
import glob
import sys


def merge(iv, tol=0):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1] + tol:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b, merged):
    tot = 0
    for s, e in merged:
        if e <= a:
            continue
        if s >= b:
            break
        tot += min(b, e) - max(a, s)
    return tot


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    for ch in "(<":
        n = n.split(ch)[0]
    return n.strip()[:40]


def main():
    d = sys.argv[1]
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        try:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                         r["Kernel_Name"]))
        except (KeyError, ValueError):
            continue
    rows.sort()
    t_end = max(r[1] for r in rows)
    t0 = rows[0][0] + int((t_end - rows[0][0]) * (1 - frac))
    rows = [r for r in rows if r[0] >= t0]
    span = t_end - t0
    pq = {r[2] for r in rows if "trunk_tail" in r[3] or "act_trunk" in r[3]}
    pol = [r for r in rows if r[2] in pq]
    lea = [r for r in rows if r[2] not in pq]
    lea_m = merge([(s, e) for s, e, _, _ in lea], tol=20_000)  # gaps < 20 us = still active
    lea_busy = sum(e - s for s, e in merge([(s, e) for s, e, _, _ in lea]))
    pol_busy = sum(e - s for s, e in merge([(s, e) for s, e, _, _ in pol]))
    all_busy = sum(e - s for s, e in merge([(s, e) for s, e, _, _ in rows]))
    starts = [i for i, r in enumerate(pol) if "decode_obs_mask" in r[3] or "act_trunk" in r[3]]
    steps = []
    for a, b in zip(starts, starts[1:]):
        s = pol[a][0]
        e = max(r[1] for r in pol[a:b])
        kb = sum(r[1] - r[0] for r in pol[a:b])
        ov = overlap(s, e, lea_m) / max(1, e - s)
        steps.append((e - s, kb, ov, pol[b][0] - e))
    act = sum(e - s for s, e in lea_m)
    print(f"window {span / 1e6:.1f} ms: GPU busy (union) {all_busy / span:.1%}; policy queue "
          f"busy {pol_busy / span:.1%}; learner queues busy {lea_busy / span:.1%}; learner active "
          f"(gaps < 20 us merged) {act / span:.1%}")
    if not steps:
        return
    inside = [x for x in steps if x[2] > 0.5]
    outside = [x for x in steps if x[2] <= 0.5]

    def stat(xs, name):
        if not xs:
            print(f"{name}: none")
            return
        n = len(xs)
        print(f"{name}: {n} steps, stream time {sum(x[0] for x in xs) / n / 1e6:.3f} ms, kernel "
              f"time {sum(x[1] for x in xs) / n / 1e6:.3f} ms, idle after "
              f"{sum(x[3] for x in xs) / n / 1e6:.3f} ms")

    stat(steps, "all policy steps")
    stat(inside, "  overlapping the learner")
    stat(outside, "  learner idle")
    # per-kernel stretch of the policy step under the learner, and which learner kernel
    # was running while the policy stream waited between two of its kernels
    names, blockers = {}, {}
    lea_sorted = sorted(lea)
    for a, b in zip(starts, starts[1:]):
        s = pol[a][0]
        e = max(r[1] for r in pol[a:b])
        ov = overlap(s, e, lea_m) / max(1, e - s) > 0.5
        for r in pol[a:b]:
            d = names.setdefault(short(r[3]), [[], []])
            d[int(ov)].append(r[1] - r[0])
        for r0, r1 in zip(pol[a:b], pol[a + 1:b]):
            gap = r1[0] - r0[1]
            if gap < 20_000:
                continue
            mid = (r0[1] + r1[0]) // 2
            for ls, le, _, ln in lea_sorted:
                if ls > mid:
                    break
                if le >= mid:
                    k = short(ln)
                    blockers[k] = blockers.get(k, 0) + gap
                    break
    print("policy kernels (mean us): learner idle | under learner")
    for k, (o, i) in sorted(names.items(), key=lambda kv: -sum(kv[1][1]) - sum(kv[1][0])):
        mo = sum(o) / len(o) / 1e3 if o else float("nan")
        mi = sum(i) / len(i) / 1e3 if i else float("nan")
        print(f"  {k:42s} {mo:8.1f} | {mi:8.1f}   (n={len(o)}|{len(i)})")
    tot = sum(blockers.values())
    print(f"policy-stream gaps > 20 us: {tot / 1e6:.1f} ms in the window; learner kernel running:")
    for k, v in sorted(blockers.items(), key=lambda kv: -kv[1])[:12]:
        print(f"  {k:42s} {v / 1e6:8.2f} ms")


if __name__ == "__main__":
    main()
