#!/usr/bin/env python3
"""Median HIP API / kernel durations per read from a rocprofv3 csv trace dir
(scripts/trace_feed.py runs).   kt_summary.py DIR [reads]"""
import collections
import csv
import statistics as st
import sys

d = sys.argv[1]
reads = int(sys.argv[2]) if len(sys.argv) > 2 else 299
for name, key in (("hip_api_trace", "Function"), ("kernel_trace", "Kernel_Name")):
    try:
        rows = list(csv.DictReader(open(f"{d}/run_{name}.csv")))
    except FileNotFoundError:
        continue
    g = collections.defaultdict(list)
    for r in rows:
        g[r[key][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        if len(v) >= reads // 2:
            print(f"{name[:6]} {k:60s} n={len(v):5d} median_us={st.median(v):7.2f} per_read_us={sum(v) / reads:7.2f}")
