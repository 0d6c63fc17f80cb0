#!/usr/bin/env python3
"""Handshake-digest measurement: hvws_encode_keys
over N conforming Sec-WebSocket-Key values (24 base64 characters), device
resident, timed with HIP events on the ctx stream; a sample is checked
against the library's host ws_encode_key.  CPU baseline: the reference
ws_encode_key (oracle/_ref, one core) over a bounded sample.

The kernel is integer-VALU-bound (two SHA-1 blocks + base64 per key); its
VALU instruction count per launch comes from a separate rocprofv3 pass
(`--pmc SQ_INSTS_VALU ... --kernel-include-regex k_encode_keys -- python
scripts/bench_keys.py`, profiles/r5_raw/keys/) and is reported against the
gfx950 issue peak by DESIGN.md, not here.  Prints one JSON line.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import libhv_amd  # noqa: E402

ALPHA = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/", dtype=np.uint8)


def main():
    n = int(os.environ.get("KEYS", str(1 << 24)))
    reps = int(os.environ.get("REPS", "5"))
    eng = libhv_amd.Engine(int(os.environ.get("HVWS_BENCH_DEVICE", "0")))
    rng = np.random.default_rng(1)
    blob = ALPHA[rng.integers(0, 64, size=(n, 24), dtype=np.uint8)]
    blob[:, 22:] = ord("=")   # base64 of a 16-byte nonce ends in "=="
    blob = np.ascontiguousarray(blob).reshape(-1)
    offs = np.arange(n, dtype=np.uint64) * 24
    lens = np.full(n, 24, dtype=np.uint32)
    dk, do, dl = eng.to_device(blob), eng.to_device(offs), eng.to_device(lens)
    acc = eng.alloc(32 * n)
    L = libhv_amd.lib()
    ms = []
    for _ in range(reps + 1):
        libhv_amd._check(L.hvws_encode_keys(eng.ctx, dk.ptr, do.ptr, dl.ptr, n, acc.ptr), "encode_keys")
        ms.append(eng.last_kernel_ms())
    k = float(np.mean(ms[1:]))
    out = acc.download(32 * n)
    L.ws_encode_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    bad = 0
    for i in range(0, n, max(1, n // 2000)):
        a = ctypes.create_string_buffer(32)
        L.ws_encode_key(blob[24 * i:24 * i + 24].tobytes(), a)
        bad += a.raw != out[32 * i:32 * i + 32].tobytes()
    res = {"bench": "encode_keys", "keys": n, "kernel_ms": round(k, 3), "keys_per_s": round(n / k * 1e3, 1),
           "GBps_io": round(n * (24 + 8 + 4 + 32) / k / 1e6, 1), "verified_sample_mismatches": int(bad)}
    try:
        import wsharness as H
        if H.have_ref():
            R = H.ref()
            R.msgp_bench_keys.restype = ctypes.c_uint64
            R.msgp_bench_keys.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p]
            m = min(n, 1 << 20)
            cbuf = np.zeros(32 * m, dtype=np.uint8)
            t = time.perf_counter()
            R.msgp_bench_keys(blob.ctypes.data, m, 24, 24, cbuf.ctypes.data)
            dt = time.perf_counter() - t
            res["cpu_baseline"] = {"keys_per_s": round(m / dt, 1), "cores": 1, "kind": "reference",
                                   "sample": f"{m} keys", "matches_gpu": bool((cbuf == out[:32 * m]).all())}
    except Exception as e:  # noqa: BLE001 -- the baseline is optional on a box without oracle/_ref
        res["cpu_baseline"] = {"error": str(e)}
    print(json.dumps(res), flush=True)
    for b in (dk, do, dl, acc):
        b.free()
    eng.close()


if __name__ == "__main__":
    main()
