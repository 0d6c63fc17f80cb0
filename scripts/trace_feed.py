#!/usr/bin/env python3
"""Per-read FeedRecvData loop for a runtime trace (design record, not a
benchmark): N 8 KiB reads of masked 1 KiB frames on one connection through
hvws_wsp_feed, timed per call.  Run under rocprofv3 --hip-runtime-trace
--kernel-trace --memory-copy-trace to see where a read's ~50 us goes."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import libhv_amd  # noqa: E402
import wsharness as H  # noqa: E402
from libhv_amd import synth  # noqa: E402

READ = 8192
n = int(os.environ.get("READS", "300"))
L = libhv_amd.lib()
plan = synth.uniform_plan(n * READ // 1032 + 2, 1024, 5)
host = np.array(H.synth_cpu(plan), copy=True)
h = L.hvws_wsp_new()
base = host.ctypes.data
L.hvws_wsp_feed(h, base, READ)   # warm-up
t = []
for i in range(1, n):
    t0 = time.perf_counter()
    L.hvws_wsp_feed(h, base + i * READ, READ)
    t.append(time.perf_counter() - t0)
t = np.array(t) * 1e6
print(f"reads={len(t)} median_us={np.median(t):.1f} p10={np.percentile(t, 10):.1f} p90={np.percentile(t, 90):.1f}")
