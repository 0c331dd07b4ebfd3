#!/usr/bin/env python
"""Per-kernel hardware-counter summary of rocprofv3 ``--pmc ... --kernel-trace`` runs.

usage: python tools/pmc_summary.py <out.md> <rocprof_dir> [<rocprof_dir> ...]

Each directory is one counter pass (rocprofv3 does not multiplex passes). Rows of the
counter CSVs are summed per dispatch and counter. Per kernel
name (aggregated over dispatches) the table reports what the counters of that kernel's
passes allow:

* MFMA util   = sum SQ_VALU_MFMA_BUSY_CYCLES / (cycles * 1024 SIMDs)
* LDS conflict = sum SQ_LDS_BANK_CONFLICT / (cycles * 256 CUs)   (% of cycles)
  with cycles = GRBM_GUI_ACTIVE / 8 (see XCDS)
* HBM GB/s    = (FETCH_SIZE + WRITE_SIZE) / kernel time (kernel-trace durations)
"""
import collections
import csv
import glob
import os
import sys

SIMDS, CUS, XCDS = 1024, 256, 8  # MI355X: 256 CUs x 4 SIMDs in 8 XCDs
# rocprofv3 writes one row per (dispatch, counter) already summed over its dimensions, so
# GRBM_GUI_ACTIVE comes out as the sum of the 8 XCDs' busy-cycle counts: / XCDS gives the
# dispatch's cycles (checked: 16.0 MFMA-busy cycles per 16x16x32 bf16 MFMA instruction and
# conv FLOP rates then agree with the kernel-trace times)


def _find(d, pat):
    return sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))


def load_pass(d):
    """-> {dispatch_id: (kernel, {counter: value})}, {dispatch_id: duration_ns}"""
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in _find(d, "*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            cn, cv = r.get("Counter_Name"), r.get("Counter_Value")
            if did is None or cn is None or cv is None:
                continue
            names[did] = r.get("Kernel_Name", "?")
            v = float(cv)
            vals[did][cn] += v
    dur = {}
    for f in _find(d, "*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            try:
                dur[did] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            except (KeyError, ValueError, TypeError):
                pass
    return {k: (names[k], dict(v)) for k, v in vals.items()}, dur


def short(n, k=78):
    n = n.replace("(anonymous namespace)::", "")
    return n if len(n) <= k else n[: k - 3] + "..."


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))  # kernel -> sums
    for d in dirs:
        disp, dur = load_pass(d)
        for did, (kn, cv) in disp.items():
            a = agg[kn]
            t = dur.get(did, 0)
            for c, v in cv.items():
                a[c] += v
                a["_t_" + c] += t  # kernel time covered by this counter's dispatches
            a["_n_" + os.path.basename(d)] += 1
    rows = []
    for kn, a in agg.items():
        t_any = max((v for k, v in a.items() if k.startswith("_t_")), default=0)
        cyc = a.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        mfma = (100.0 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS)
                if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in a else None)
        lds = (100.0 * a["SQ_LDS_BANK_CONFLICT"] / (cyc * CUS)
               if cyc and "SQ_LDS_BANK_CONFLICT" in a else None)
        bw = None
        if "FETCH_SIZE" in a and "WRITE_SIZE" in a and a.get("_t_FETCH_SIZE") and a.get("_t_WRITE_SIZE"):
            bw = (a["FETCH_SIZE"] * 1024 / a["_t_FETCH_SIZE"] + a["WRITE_SIZE"] * 1024 / a["_t_WRITE_SIZE"])
        insts = a.get("SQ_INSTS_MFMA")
        per = (a["SQ_VALU_MFMA_BUSY_CYCLES"] / insts
               if insts and "SQ_VALU_MFMA_BUSY_CYCLES" in a else None)
        rows.append((t_any, kn, mfma, lds, bw, insts, per))
    rows.sort(key=lambda r: -r[0])
    fmt = lambda v, f: "-" if v is None else f.format(v)  # noqa: E731
    lines = ["| kernel | kernel ms (pass) | MFMA util % | MFMA insts (M) | busy cyc / MFMA | "
             "LDS bank-conflict % | HBM GB/s |",
             "|---|---|---|---|---|---|---|"]
    for t, kn, mfma, lds, bw, insts, per in rows[:30]:
        lines.append(f"| `{short(kn)}` | {t / 1e6:.2f} | {fmt(mfma, '{:.1f}')} | "
                     f"{fmt(insts and insts / 1e6, '{:.1f}')} | {fmt(per, '{:.1f}')} | "
                     f"{fmt(lds, '{:.1f}')} | {fmt(bw, '{:.0f}')} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
