#!/usr/bin/env python
"""Offline smoothing of an episode CSV into 10-episode means.

Reference: data_processor.py (interactive prompt, writes ``{name}_processed.csv``
with rows [window, mean_return, mean_steps]; its remainder row dropped the
window index). Non-interactive here (``--name``), same output file, the
remainder row keeps its index.

    python tools/process_csv.py --name runs/exp1 [--window 10]
"""
from __future__ import annotations

import argparse
import csv


def process(name: str, window: int = 10) -> str:
    src, dst = f"{name}.csv", f"{name}_processed.csv"
    with open(src) as f:
        rows = list(csv.reader(f))
    header, body = rows[0], [r for r in rows[1:] if r]
    out = []
    for w, i in enumerate(range(0, len(body), window)):
        chunk = body[i:i + window]
        rets = [float(r[0]) for r in chunk]
        steps = [float(r[1]) for r in chunk]
        out.append([w, sum(rets) / len(rets), sum(steps) / len(steps)])
    with open(dst, "w", newline="") as f:
        wr = csv.writer(f)
        wr.writerow(header[:2])
        wr.writerows(out)
    return dst


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--name", required=True, help="CSV path without .csv")
    p.add_argument("--window", type=int, default=10)
    a = p.parse_args(argv)
    print(process(a.name, a.window))


if __name__ == "__main__":
    main()
