#!/usr/bin/env python
"""Learning-curve summary of a training run's CSVs (rank-0 ``{exp}.csv`` episodes and
``{exp}Losses.csv``), for committing evidence that a run learned.

Writes ``{name}_processed.csv`` (reference data_processor.py format: window index, mean
return, mean steps; ``--window`` episodes per row, default 10 like the reference) and
``{name}_curve.md`` (per-segment mean return / win / loss / draw rates / episode length,
plus the loss columns at matching updates); optionally gzips the raw episode CSV.

    python tools/learning_curve.py --name runs/exp8/exp8 [--segments 10] [--window 1000]
"""
from __future__ import annotations

import argparse
import csv
import gzip
import os
import shutil


def summarize(name: str, segments: int = 10, window: int = 10, gz: bool = False) -> str:
    with open(f"{name}.csv") as f:
        eps = list(csv.DictReader(f))
    losses = []
    if os.path.exists(f"{name}Losses.csv"):
        with open(f"{name}Losses.csv") as f:
            losses = list(csv.DictReader(f))
    n = len(eps)
    proc = f"{name}_processed.csv"
    with open(proc, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Return", "steps"])
        for k, i in enumerate(range(0, n, window)):
            ch = eps[i:i + window]
            w.writerow([k, round(sum(float(e["Return"]) for e in ch) / len(ch), 4),
                        round(sum(float(e["steps"]) for e in ch) / len(ch), 2)])
    lines = [f"# Learning curve: `{os.path.basename(name)}`", "",
             f"{n} finished episodes, {len(losses)} logged updates.", "",
             "| episodes | mean return | win | loss | draw/timeout | mean length |",
             "|---|---|---|---|---|---|"]
    k = max(1, n // segments)
    for i in range(0, n, k):
        ch = eps[i:i + k]
        if len(ch) < k // 2:
            break
        m = len(ch)
        ret = sum(float(e["Return"]) for e in ch) / m
        win = sum(e.get("winner") == "0" for e in ch) / m
        loss = sum(e.get("winner") == "1" for e in ch) / m
        ln = sum(float(e["steps"]) for e in ch) / m
        lines.append(f"| {i}-{i + m - 1} | {ret:.2f} | {win:.3f} | {loss:.3f} | "
                     f"{1 - win - loss:.3f} | {ln:.1f} |")
    if losses:
        lines += ["", "| update | frames | pg_loss | value_loss | entropy | fps | policy_lag |",
                  "|---|---|---|---|---|---|---|"]
        kk = max(1, len(losses) // segments)
        for r in losses[::kk] + ([losses[-1]] if (len(losses) - 1) % kk else []):
            lines.append(f"| {r['update']} | {r.get('frames', '')} | {float(r['pg_loss']):.4f} | "
                         f"{float(r['value_loss']):.4f} | {float(r['entropy_loss']):.4f} | "
                         f"{float(r.get('fps') or 0):,.0f} | {r.get('policy_lag', '')} |")
    md = f"{name}_curve.md"
    with open(md, "w") as f:
        f.write("\n".join(lines) + "\n")
    if gz:
        with open(f"{name}.csv", "rb") as src, gzip.open(f"{name}.csv.gz", "wb") as dst:
            shutil.copyfileobj(src, dst)
        os.remove(f"{name}.csv")
    return md


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--name", required=True, help="run prefix: <savedir>/<exp_name>")
    p.add_argument("--segments", type=int, default=10)
    p.add_argument("--window", type=int, default=10)
    p.add_argument("--gzip", action="store_true", help="replace the raw episode CSV by .csv.gz")
    a = p.parse_args(argv)
    print(summarize(a.name, a.segments, a.window, a.gzip))


if __name__ == "__main__":
    main()
