#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats / kernel trace / PMC counters)
into a small markdown table for profiles/.

  scripts/prof_summary.py <rocprof dir> [--pmc-dir DIR ...] > profiles/rNN_x.md
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def short(name: str) -> str:
    name = name.split("(")[0]
    return name.replace("void ", "").replace("hvws::", "")


def kernel_stats(d: str):
    rows = []
    for f in glob.glob(os.path.join(d, "*kernel_stats.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                             float(r["Percentage"]), float(r["MinNs"]), float(r["MaxNs"])))
    return rows


def counters(d: str):
    """{kernel: {counter: [values per dispatch]}}"""
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                out[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--pmc-dir", action="append", default=[])
    ap.add_argument("--title", default="rocprofv3 --kernel-trace --stats")
    a = ap.parse_args()
    print(f"## {a.title}\n")
    print("| kernel | calls | total ms | avg us | % | min us | max us |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for n, c, tot, avg, pct, mn, mx in sorted(kernel_stats(a.trace_dir), key=lambda r: -r[2]):
        print(f"| `{n}` | {c} | {tot / 1e6:.3f} | {avg / 1e3:.1f} | {pct:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} |")
    for d in a.pmc_dir:
        cs = counters(d)
        if not cs:
            continue
        print(f"\n### PMC ({os.path.basename(d.rstrip('/'))}), median per dispatch\n")
        names = sorted({c for k in cs.values() for c in k})
        print("| kernel | dispatches | " + " | ".join(names) + " |")
        print("|---|---:|" + "---:|" * len(names))
        for k, m in sorted(cs.items()):
            nd = max(len(v) for v in m.values())
            vals = [f"{statistics.median(m[c]):.4g}" if c in m else "" for c in names]
            print(f"| `{k}` | {nd} | " + " | ".join(vals) + " |")


if __name__ == "__main__":
    main()
