#!/usr/bin/env python3
"""Transmit-side measurement: hvws_build_frames
over the config-3 shape (1M masked binary frames x 64 KiB), device resident.

Two payload layouts:
  * "rx_layout": the payloads sit where the receive path left them (the
    unmasked rx batch) -- payload and output 16-B phases agree;
  * "packed": payloads back to back in a send arena -- every 64 KiB frame's
    14-byte header shifts the output phase, so loads are realigned.
Both layouts build from real payload bytes and every output byte is checked
against the masked batch.  Algorithmic bytes per launch = payload read +
frames written.  Device time from HIP events around the call's device work
after its size check (tile index and spans when the layout needs them, and
k_build) on the ctx stream.  Prints JSON lines.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import libhv_amd  # noqa: E402
from libhv_amd import synth  # noqa: E402

PEAK = 8000.0


def main():
    reps = int(os.environ.get("REPS", "5"))
    name = os.environ.get("CONFIG", "c3")
    eng = libhv_amd.Engine(int(os.environ.get("HVWS_BENCH_DEVICE", "0")))
    L = libhv_amd.lib()
    p = synth.config_plan(name, 1).split(4096)
    dp = libhv_amd.DevicePlan(eng, p)
    hdr = synth.frame_size(p.flags, p.length) - p.length
    rx = eng.alloc(p.total + 64)
    out = eng.alloc(p.total + 64)
    eng.synth(rx, p.total, p.seed, dp, 0)
    eng.step(rx, p.total, p.segments)
    eng.sync()
    alg = p.payload_bytes + p.total
    pack_off = np.concatenate([[0], np.cumsum(p.length)[:-1]]).astype(np.uint64)
    # a real packed send arena: every frame's plaintext payload back to back,
    # compacted on the host out of the unmasked rx batch
    host = rx.download(p.total)
    packed = np.empty(max(p.payload_bytes, 1), dtype=np.uint8)
    src = (p.frame_off + hdr).astype(np.int64)
    if len(set(np.unique(p.length).tolist())) == 1 and np.all(np.diff(src) == src[1] - src[0] if p.n > 1 else True):
        ln, st = int(p.length[0]), int(src[1] - src[0]) if p.n > 1 else 0
        view = np.lib.stride_tricks.as_strided(host[int(src[0]):], shape=(p.n, ln), strides=(st, 1))
        packed[:p.payload_bytes] = view.reshape(-1)
    else:
        for k in range(p.n):
            o, ln = int(pack_off[k]), int(p.length[k])
            packed[o:o + ln] = host[src[k]:src[k] + ln]
    del host
    arena = eng.to_device(packed)
    del packed
    for layout, offs, pay in (("rx_layout", p.frame_off + hdr, rx), ("packed", pack_off, arena)):
        tx = libhv_amd.TxPlan(eng, offs, p.length, p.flags, p.mask)
        ms = []
        t0 = time.perf_counter()
        plen = p.total if pay is rx else p.payload_bytes
        for _ in range(reps + 1):
            n = eng.build_frames(out, p.total + 64, pay, plen, tx)
            ms.append(eng.last_kernel_ms())
        wall = (time.perf_counter() - t0) / (reps + 1)
        assert n == p.total
        # every output byte against the masked batch (device synth VERIFY)
        ok = eng.synth(out, p.total, p.seed, dp, 1) == 0
        L.hvws_memset(eng.ctx, out.ptr, 0, p.total)   # the next layout must write every byte itself
        k = float(np.mean(ms[1:]))
        print(json.dumps({
            "bench": "build_frames", "kernel": libhv_amd.lib().hvws_last_build_kernel(eng.ctx).decode(), "config": name,
            "index": "none (uniform layout)" if L.hvws_last_build_uniform(eng.ctx) else "tile index + spans",
            "layout": layout, "frames": p.n,
            "payload_bytes": p.payload_bytes, "out_bytes": p.total, "alg_bytes_per_launch": alg,
            "kernel_ms": round(k, 3), "kernel_GBps": round(alg / k / 1e6, 1),
            "frac_of_8TBps": round(alg / k / 1e6 / PEAK, 4),
            "call_ms": round(wall * 1e3, 3), "payload_GiBps_call": round(p.payload_bytes / wall / 2**30, 1),
            "verified": ok,
        }), flush=True)
        tx.free()
        if not ok:
            raise SystemExit(f"{layout}: the built frames differ from the masked batch")
    arena.free()
    # ceilings: runtime D2D copy of the same bytes, and one huge unmasked frame
    # (k_build's streaming path as a plain realigning copy)
    ev = []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        L.hvws_d2d(eng.ctx, out.ptr, rx.ptr, p.payload_bytes)
        eng.sync()
        ev.append(time.perf_counter() - t0)
    d2d = float(np.mean(ev[1:]))
    one = libhv_amd.TxPlan(eng, [0], [p.payload_bytes], [0x12], [0])
    ms = []
    for _ in range(reps + 1):
        eng.build_frames(out, p.total + 64, rx, p.total, one)
        ms.append(eng.last_kernel_ms())
    k1 = float(np.mean(ms[1:]))
    one.free()
    print(json.dumps({"bench": "copy_ceiling", "bytes_moved": 2 * p.payload_bytes,
                      "d2d_GBps_wall": round(2 * p.payload_bytes / d2d / 1e9, 1),
                      "one_frame_build_GBps": round((2 * p.payload_bytes + 10) / k1 / 1e6, 1)}), flush=True)
    rx.free()
    out.free()
    dp.free()
    eng.close()


if __name__ == "__main__":
    main()
