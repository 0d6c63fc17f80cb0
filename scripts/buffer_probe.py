#!/usr/bin/env python3
"""Design probe (not product code): is the in-place stream rate a property of
the box or of the buffer?  Three 64 GiB buffers allocated one after another,
the in-place STREAM kernel (hvws_stream_xor, the c3 geometry) timed on each,
interleaved over rounds; prints GB/s per buffer as one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhv_amd  # noqa: E402

eng = libhv_amd.Engine(0)
n = 64 << 30
bufs = []
for i in range(3):
    b = eng.alloc(n)
    libhv_amd._check(libhv_amd.lib().hvws_memset(eng.ctx, b.ptr, i, n), "memset")
    bufs.append(b)
eng.sync()
rates = {i: [] for i in range(3)}
for r in range(6):
    for i, b in enumerate(bufs):
        eng.sync()
        t = time.perf_counter()
        eng.stream_xor(b, n, 0x5A5A5A5A)
        eng.stream_xor(b, n, 0x5A5A5A5A)
        eng.sync()
        if r:
            rates[i].append(2 * 2 * n / (time.perf_counter() - t) / 1e9)
print(json.dumps({"GBps_median": {f"buf{i}": round(float(np.median(v)), 1) for i, v in rates.items()},
                  "GBps_all": {f"buf{i}": [round(x, 1) for x in v] for i, v in rates.items()},
                  "kernel": libhv_amd.lib().hvws_unmask_kernel_name_for(n).decode()}))
