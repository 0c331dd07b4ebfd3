#!/usr/bin/env python
"""Raw per-kernel counter totals (and per-wave / per-cycle ratios) of rocprofv3 --pmc passes.

usage: python tools/pmc_raw.py <filter substring> <rocprof_dir> [<rocprof_dir> ...]
"""
import collections
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from pmc_summary import load_pass  # noqa: E402


def main():
    filt = sys.argv[1]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    durs = collections.defaultdict(float)
    for d in sys.argv[2:]:
        vals, dur = load_pass(d)
        for did, (name, cv) in vals.items():
            if filt not in name:
                continue
            key = name.replace("(anonymous namespace)::", "").split("(")[0][:60]
            cnt[key] += 1
            durs[key] += dur.get(did, 0)
            for c, v in cv.items():
                tot[key][c] += v
    for k, cv in tot.items():
        print(f"== {k}: {cnt[k]} dispatch-passes, kernel time {durs[k] / 1e6:.3f} ms (summed over passes)")
        waves = cv.get("SQ_WAVES", 0)
        for c in sorted(cv):
            extra = f"  per-wave {cv[c] / waves:.1f}" if waves else ""
            print(f"   {c:28s} {cv[c]:16.0f}{extra}")


if __name__ == "__main__":
    main()
