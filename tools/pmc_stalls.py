"""Per-kernel sums of the counters in one or more rocprofv3 --pmc output dirs (stall study).

    python tools/pmc_stalls.py <out.md> <dir> [<dir> ...] [--match substr,substr]
"""
import collections
import csv
import glob
import os
import sys


def main():
    out, dirs = sys.argv[1], [d for d in sys.argv[2:] if not d.startswith("--")]
    match = []
    for a in sys.argv[2:]:
        if a.startswith("--match="):
            match = a.split("=", 1)[1].split(",")
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "")
                if match and not any(m in k for m in match):
                    continue
                k = k.replace("(anonymous namespace)::", "")[:70]
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((d, r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
    names = sorted({c for v in tot.values() for c in v})
    with open(out, "w") as fo:
        fo.write("| kernel | dispatches | " + " | ".join(names) + " |\n")
        fo.write("|---" * (len(names) + 2) + "|\n")
        for k, v in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
            fo.write(f"| `{k}` | {len(disp[k])} | " + " | ".join(f"{v.get(c, 0):.4g}" for c in names) + " |\n")
    print(open(out).read())


if __name__ == "__main__":
    main()
