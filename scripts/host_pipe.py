#!/usr/bin/env python3
"""Host-inclusive rate (hvws_pipeline) against chunk size (design probe).

Builds config-3 frames (64 KiB) in pinned host memory, then runs
hvws_pipeline over them with several chunk sizes, each repeated, and prints
wire GB/s per chunk size as JSON lines (the bytes are unmasked and masked
again on alternate runs).  The link's own concurrent H2D+D2H rate with the
same piece size is printed beside it.

  scripts/host_pipe.py [--gib 4] [--chunks-mib 16,64,256] [--reps 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libhv_amd  # noqa: E402
from libhv_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--chunks-mib", default="16,32,64,128,256")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import bench  # pcie_ceiling

    L = libhv_amd.lib()
    eng = libhv_amd.Engine(0)
    n = int(a.gib * (1 << 30) / 65550)
    plan = synth.uniform_plan(n, 65536, 5)
    dp = libhv_amd.DevicePlan(eng, plan)
    rx = eng.alloc(plan.total + 64)
    eng.synth(rx, plan.total, plan.seed, dp, 0)
    pinned = L.hvws_host_alloc(eng.ctx, plan.total)
    libhv_amd._check(L.hvws_d2h(eng.ctx, pinned, rx.ptr, plan.total), "d2h")
    eng.sync()
    rx.free()
    dp.free()
    for cm in [int(x) for x in a.chunks_mib.split(",")]:
        chunk = cm << 20
        rates = []
        for _ in range(a.reps):
            carry = libhv_amd.WsParser()
            L.websocket_parser_init(ctypes.byref(carry))
            t = time.perf_counter()
            libhv_amd._check(L.hvws_pipeline(eng.ctx, pinned, plan.total, chunk, ctypes.byref(carry)), "pipeline")
            rates.append(plan.total / (time.perf_counter() - t) / 1e9)
        link = bench.pcie_ceiling(0, piece=chunk)
        print(json.dumps({"chunk_mib": cm, "bytes": plan.total, "GBps_wire": [round(r, 2) for r in rates],
                          "link": link}), flush=True)
    L.hvws_host_free(eng.ctx, pinned)
    eng.close()


if __name__ == "__main__":
    main()
