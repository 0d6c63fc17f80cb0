#!/usr/bin/env python3
"""Per-step timeline from a rocprofv3 --kernel-trace CSV: for each k_unmask
dispatch (one per bench step) list the kernels since the previous one with
their durations and the idle gap before each, then the step's wall time
(unmask end to unmask end), busy time and idle time.

  scripts/trace_gaps.py <rocprof dir> [--steps N] [--detail]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").replace("hvws::", "")


def load(d: str):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--detail", action="store_true")
    a = ap.parse_args()
    rows = load(a.trace_dir)
    ends = [i for i, r in enumerate(rows) if r[2].startswith("k_unmask")]
    if len(ends) < 2:
        print("fewer than two k_unmask dispatches")
        return
    print("| step | wall ms | kernels | busy ms | idle ms | unmask ms | scan-side busy ms |")
    print("|---:|---:|---:|---:|---:|---:|---:|")
    sel = list(zip(ends[:-1], ends[1:]))[-a.steps:]
    for n, (i0, i1) in enumerate(sel):
        seg = rows[i0 + 1:i1 + 1]
        wall = (rows[i1][1] - rows[i0][1]) / 1e6
        busy = sum(e - s for s, e, _ in seg) / 1e6
        um = (rows[i1][1] - rows[i1][0]) / 1e6
        print(f"| {n} | {wall:.3f} | {len(seg)} | {busy:.3f} | {wall - busy:.3f} | {um:.3f} | {busy - um:.3f} |")
    if a.detail:
        i0, i1 = sel[-1]
        print("\n| kernel | start us | dur us | gap before us |")
        print("|---|---:|---:|---:|")
        prev = rows[i0][1]
        t0 = rows[i0][1]
        for s, e, k in rows[i0 + 1:i1 + 1]:
            print(f"| `{k}` | {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {(s - prev) / 1e3:.1f} |")
            prev = e


if __name__ == "__main__":
    main()
