#!/usr/bin/env python
"""Does anything serialize behind the collective stream? (bench.py --comm_rehearsal trace)

usage: python tools/rehearsal_trace.py <rocprof_out_dir> [<baseline_rocprof_out_dir>]

Reads a rocprofv3 --kernel-trace CSV of ``bench.py --comm_rehearsal`` (world 1: every
gradient bucket fires ``comm_standin_kernel`` on a 4th, high-priority stream from the grad
hooks, parallel/dist.py) and reports, over the second half of the run:

* the hardware queues the three kinds of work landed on (policy lanes: act_trunk / head_act
  / trunk_tail; collective: comm_standin; learner: the rest). A shared queue id between the
  collective and a lane or the learner would serialize them;
* per stand-in kernel, the share of its run time during which learner / policy kernels ran
  concurrently (they overlap rather than wait);
* the policy step's kernel times while a stand-in runs vs not, and the learner's exposed wait:
  from the last backward kernel before the optimizer to the end of the update's last stand-in.

With a baseline directory (the same bench without --comm_rehearsal) it also compares the
policy kernels' mean durations.
"""
import csv
import glob
import sys


def load(d):
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
    t0 = rows[0][0] + (t_end - rows[0][0]) // 2
    return [r for r in rows if r[0] >= t0]


def kind(name):
    if "comm_standin" in name:
        return "comm"
    if "act_trunk" in name or "head_act" in name or "trunk_tail" in name:
        return "policy"
    return "learner"


def merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(a, b, merged):
    tot = 0
    for s, e in merged:
        if e <= a:
            continue
        if s >= b:
            break
        tot += min(b, e) - max(a, s)
    return tot


def policy_means(rows):
    out = {}
    for s, e, _, n in rows:
        if kind(n) == "policy":
            k = "act_trunk" if "act_trunk" in n else "head_act" if "head_act" in n else "trunk_tail"
            out.setdefault(k, []).append(e - s)
    return {k: sum(v) / len(v) / 1e3 for k, v in out.items()}


def main():
    rows = load(sys.argv[1])
    queues = {}
    for _, _, q, n in rows:
        queues.setdefault(kind(n), set()).add(q)
    print("hardware queues:", {k: sorted(v) for k, v in queues.items()})
    shared = {(a, b): queues.get(a, set()) & queues.get(b, set())
              for a, b in (("comm", "policy"), ("comm", "learner"), ("policy", "learner"))}
    for (a, b), s in shared.items():
        print(f"  {a} / {b} share queue(s): {sorted(s) if s else 'none'}")
    comm = [r for r in rows if kind(r[3]) == "comm"]
    if not comm:
        print("no comm_standin kernels in the window (not a --comm_rehearsal run?)")
        return
    lea = merge([(s, e) for s, e, _, n in rows if kind(n) == "learner"])
    pol = merge([(s, e) for s, e, _, n in rows if kind(n) == "policy"])
    cm = merge([(s, e) for s, e, _, _ in comm])
    tot = sum(e - s for s, e, _, _ in comm)
    print(f"{len(comm)} stand-in kernels, mean {tot / len(comm) / 1e3:.1f} us; concurrent with "
          f"learner kernels {sum(covered(s, e, lea) for s, e, _, _ in comm) / tot:.1%}, with "
          f"policy kernels {sum(covered(s, e, pol) for s, e, _, _ in comm) / tot:.1%} of their time")
    # policy kernels while a stand-in runs vs not
    during, outside = {}, {}
    for s, e, _, n in rows:
        if kind(n) != "policy":
            continue
        k = "act_trunk" if "act_trunk" in n else "head_act" if "head_act" in n else "trunk_tail"
        d = during if covered(s, e, cm) > 0.5 * (e - s) else outside
        d.setdefault(k, []).append(e - s)
    print("policy kernels (mean us): no stand-in running | stand-in running")
    for k in sorted(set(during) | set(outside)):
        o, i = outside.get(k, []), during.get(k, [])
        print(f"  {k:12s} {sum(o) / max(1, len(o)) / 1e3:8.1f} | {sum(i) / max(1, len(i)) / 1e3:8.1f}"
              f"   (n={len(o)}|{len(i)})")
    # learner exposure: per update, the optimizer kernel's start minus the last learner kernel
    # before it, when a stand-in ended in that gap
    lrows = [r for r in rows if kind(r[3]) == "learner"]
    waits = []
    for i, (s, e, q, n) in enumerate(lrows):
        if "adam" not in n.lower() or i == 0:
            continue
        prev_end = max(r[1] for r in lrows[max(0, i - 8):i])
        last_comm = max((c[1] for c in comm if c[1] <= s and c[1] >= prev_end - 50_000_000),
                        default=None)
        if last_comm is not None and last_comm > prev_end:
            waits.append(last_comm - prev_end)
        else:
            waits.append(0)
    if waits:
        print(f"learner wait for the collective stream before the optimizer: mean "
              f"{sum(waits) / len(waits) / 1e3:.1f} us over {len(waits)} updates "
              f"(max {max(waits) / 1e3:.1f} us)")
    if len(sys.argv) > 2:
        a, b = policy_means(load(sys.argv[2])), policy_means(rows)
        print("policy kernel means (us): baseline | rehearsal")
        for k in sorted(set(a) | set(b)):
            print(f"  {k:12s} {a.get(k, float('nan')):8.1f} | {b.get(k, float('nan')):8.1f}")


if __name__ == "__main__":
    main()
