"""Probe for the round-3 hang: the bench's drop-in
leg (FeedRecvData through the resident worker on the thread context, worker
toggled on/off) followed by host-inclusive work on another context
(hvws_host_alloc + hvws_pipeline + hvws_host_free), repeated.  Prints one
line per round with its timings, flushed, so a stuck round is visible."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import libhv_amd  # noqa: E402
from libhv_amd import synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
L = libhv_amd.lib()
with libhv_amd.Engine(0) as eng:
    fp = synth.uniform_plan(4096, 1024, 7)
    dp = libhv_amd.DevicePlan(eng, fp)
    b = eng.alloc(fp.total + 64)
    eng.synth(b, fp.total, fp.seed, dp, 0)
    feed = b.download(fp.total)
    b.free()
    dp.free()
    hp = synth.uniform_plan(4100, 65536, 3)   # 268.7 MB of 64 KiB frames
    hbytes = 256 << 20
    hdp = libhv_amd.DevicePlan(eng, hp)
    rx = eng.alloc(hp.total + 64)
    eng.synth(rx, hp.total, hp.seed, hdp, 0)
    for r in range(rounds):
        t0 = time.perf_counter()
        buf = ctypes.create_string_buffer(feed.tobytes(), len(feed))
        for mode in (1, 0, 1):
            L.hvws_set_door(None, mode)
            h = L.hvws_wsp_new()
            for i in range(200):
                assert L.hvws_wsp_feed(h, ctypes.addressof(buf) + (i % 400) * 8192, 8192) == 8192
            L.hvws_wsp_free(h)
        L.hvws_set_door(None, 0 if r % 2 else 1)
        t1 = time.perf_counter()
        pinned = L.hvws_host_alloc(eng.ctx, hbytes)
        assert L.hvws_d2h(eng.ctx, pinned, rx.ptr, hbytes) == 0
        eng.sync()
        carry = libhv_amd.WsParser()
        L.websocket_parser_init(ctypes.byref(carry))
        rc = L.hvws_pipeline(eng.ctx, pinned, hbytes, 64 << 20, ctypes.byref(carry))
        L.hvws_host_free(eng.ctx, pinned)
        t2 = time.perf_counter()
        st = (ctypes.c_uint64 * 4)()
        L.hvws_door_stats(None, st)
        print(f"round {r}: feed {1e3 * (t1 - t0):.1f} ms, host_alloc+pipeline+free {1e3 * (t2 - t1):.1f} ms, "
              f"rc {rc}, door stats {list(st)}", flush=True)
    rx.free()
    hdp.free()
print("done", flush=True)
