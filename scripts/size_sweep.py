#!/usr/bin/env python3
"""Unmask geometry against batch size (design probe, not product code).

For uniform 64 KiB-frame batches of several sizes, times k_unmask under each
of a few geometries (hvws_set_unmask_variant), interleaved round by round,
and prints the median algorithmic GB/s per (size, geometry) as JSON lines.

  scripts/size_sweep.py [--sizes-gib 0.25,1,4,16,64] [--variants 0,9,11] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libhv_amd  # noqa: E402
from libhv_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-gib", default="0.25,1,4,16,64")
    ap.add_argument("--variants", default="0,9,11")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frame", type=int, default=65536)
    a = ap.parse_args()
    L = libhv_amd.lib()
    variants = [int(v) for v in a.variants.split(",")]
    eng = libhv_amd.Engine(0)
    for gib in [float(x) for x in a.sizes_gib.split(",")]:
        n = max(1, int(gib * (1 << 30) / a.frame))
        plan = synth.uniform_plan(n, a.frame, 7).split(min(4096, n))
        dp = libhv_amd.DevicePlan(eng, plan)
        rx = eng.alloc(plan.total + 64)
        eng.synth(rx, plan.total, plan.seed, dp, 0)
        eng.sync()
        segs = eng.prepare(plan.segments)
        alg = 2 * plan.masked_payload_bytes() + plan.header_bytes
        times = {v: [] for v in variants}
        for r in range(a.rounds + 1):
            for v in variants:
                L.hvws_set_unmask_variant(v)
                eng.step(rx, plan.total, segs)
                eng.step(rx, plan.total, segs)   # even: bytes restored
                eng.sync()
                if r:
                    times[v] += [t[1] for t in eng.step_times(2)]
        names = {}
        for v in variants:
            L.hvws_set_unmask_variant(v)
            names[v] = L.hvws_unmask_kernel_name().decode()
        L.hvws_set_unmask_variant(-1)
        out = {"gib": gib, "frames": n, "alg_bytes": alg,
               "GBps": {names[v]: round(alg / (float(np.median(times[v])) * 1e-3) / 1e9, 1) for v in variants}}
        print(json.dumps(out), flush=True)
        dp.free()
        rx.free()
    eng.close()


if __name__ == "__main__":
    main()
