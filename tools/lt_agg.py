"""Aggregate a tools/layer_times.py per-dispatch table by kernel name (total us, count).
    python tools/lt_agg.py gpurun_out/x_lt.md [other.md]   (two files: side by side)"""
import collections
import sys


def agg(path):
    out = collections.OrderedDict()
    for line in open(path):
        if not (line.startswith("| ") and line[2].isdigit()):
            continue
        p = [x.strip() for x in line.split("|")]
        t = out.setdefault(p[4].strip("`"), [0.0, 0])
        t[0] += float(p[3])
        t[1] += 1
    return out


a = agg(sys.argv[1])
b = agg(sys.argv[2]) if len(sys.argv) > 2 else None
keys = list(a) + ([k for k in b if k not in a] if b else [])
keys.sort(key=lambda k: -a.get(k, [0, 0])[0])
for k in keys:
    ta, na = a.get(k, [0.0, 0])
    row = f"{ta:9.1f} {na:3d}"
    if b is not None:
        tb, nb = b.get(k, [0.0, 0])
        row += f" | {tb:9.1f} {nb:3d}"
    print(row, k)
print(f"{sum(v[0] for v in a.values()):9.1f} total" +
      (f" | {sum(v[0] for v in b.values()):9.1f}" if b else ""))
