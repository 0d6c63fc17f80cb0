#!/usr/bin/env python3
"""Event-loop shaped measurement of the drop-in.

n connections each deliver 8 KiB reads (event/hevent.h:16 HLOOP_READ_BUFSIZE)
of a stream of masked 1 KiB binary frames.  One "poll iteration" hands every
connection's next read to the parser:
  * gpu_many : one hvws_wsp_feed_many call (one GPU round trip per iteration);
  * gpu_pipe : one hvws_wsp_feeder_submit per iteration (pipelined: iteration
               k's GPU round trip overlaps iteration k-1's callback replay;
               the final flush is inside the timed region);
  * *_pinned : the connections' read buffers are slices of one pinned arena
               (hvws_host_alloc), so the reads go to the device in place
               (hvws_rx_reads: no gather into / write-back from a stage);
               connection-major (each connection's stream contiguous);
  * *_ring   : the same, iteration-major (one poll iteration's reads side by
               side, as a ring of read buffers);
  * gpu_each : WebSocketParser::FeedRecvData per connection (a round trip each);
  * cpu_ref  : the reference frame parser + restated WebSocketParser callbacks
               (oracle/_ref), per connection, one core.
  * *_general: the same through the general COUNT/EMIT/unmask sequence
               (small-batch single-launch path disabled).
Reports per-iteration latency and payload throughput.  Prints JSON lines.
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
import wsharness as H  # noqa: E402
from libhv_amd import synth  # noqa: E402

READ = 8192


def main():
    iters = int(os.environ.get("ITERS", "20"))
    L = libhv_amd.lib()
    R = H.ref() if H.have_ref() else H.oracle()
    kind = "reference" if H.have_ref() else "port"
    conns = [int(x) for x in os.environ.get("CONNS", "1,16,256,1024,4096").split(",")]
    modes = os.environ.get("MODES", "gpu_many,gpu_pipe,gpu_each,gpu_many_general,gpu_each_general,cpu_ref").split(",")
    eng = libhv_amd.Engine(0) if any(m.endswith(("_pinned", "_ring")) for m in modes) else None
    for n in conns:
        per_conn = READ * iters
        frames = per_conn // 1032 + 2
        plan = synth.uniform_plan(frames * n, 1024, 77).split(n)
        host = H.synth_cpu(plan)
        streams = [host[o:o + ln] for o, ln in plan.segments]
        payload_per_read = READ * 1024 / 1032
        res = {"connections": n, "read_bytes": READ, "iterations": iters}
        for mode in modes:
            if mode.startswith("gpu_each") and n > 256:
                continue
            # *_general: the COUNT/EMIT/unmask sequence instead of the single-launch small-batch kernel
            L.hvws_set_small_batch_limit(None, (1 << 64) - 1 if mode.endswith("_general") else 0)
            bufs = [np.array(s[:per_conn], copy=True) for s in streams]
            arena = None
            ring = mode.endswith("_ring")
            if mode.endswith("_pinned") or ring:
                # _pinned: connection i's whole stream at arena + i * per_conn;
                # _ring: iteration-major, the reads of one poll iteration side by
                # side (read `it` of connection i at arena + (it * n + i) * READ)
                arena = L.hvws_host_alloc(eng.ctx, n * per_conn)
                whole = np.ctypeslib.as_array((ctypes.c_uint8 * (n * per_conn)).from_address(arena))
                for i in range(n):
                    if ring:
                        for it in range(iters):
                            whole[(it * n + i) * READ:(it * n + i + 1) * READ] = bufs[i][it * READ:(it + 1) * READ]
                    else:
                        whole[i * per_conn:(i + 1) * per_conn] = bufs[i]
                if not ring:
                    bufs = [whole[i * per_conn:(i + 1) * per_conn] for i in range(n)]
            if mode == "cpu_ref":
                hs = [R.msgp_new() for _ in range(n)]
                t0 = time.perf_counter()
                for it in range(iters):
                    for i in range(n):
                        R.msgp_feed(hs[i], bufs[i].ctypes.data + it * READ, READ)
                dt = time.perf_counter() - t0
                for h in hs:
                    R.msgp_free(h)
            else:
                hs = [L.hvws_wsp_new() for _ in range(n)]
                hv = (ctypes.c_void_p * n)(*hs)
                lens = (ctypes.c_size_t * n)(*([READ] * n))
                rets = (ctypes.c_int * n)()
                ds = (ctypes.c_void_p * n)()
                # read pointers for iteration `it` = base + it * READ, set in one
                # numpy add (a per-connection Python loop would add ~0.5 us each)
                if ring:
                    base = np.array([arena + i * READ for i in range(n)], dtype=np.uint64)
                    step = n * READ
                else:
                    base = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
                    step = READ
                ds_np = np.frombuffer(ds, dtype=np.uint64)
                # warm-up iteration on a scratch copy (allocations, first launch)
                scratch = [np.array(b[:READ], copy=True) for b in bufs]   # pageable: the warm-up takes the staging path
                for i in range(n):
                    ds[i] = scratch[i].ctypes.data
                warm = [L.hvws_wsp_new() for _ in range(n)]
                # gpu_pipe_inline: runs <= 256 KiB do their device half on the loop thread
                os.environ["HVWS_EXPERIMENT"] = "feeder_inline=" + (str(256 << 10) if mode == "gpu_pipe_inline" else "0")
                feeder = L.hvws_feeder_new() if mode.startswith("gpu_pipe") else None
                if feeder:
                    L.hvws_wsp_feeder_submit(feeder, (ctypes.c_void_p * n)(*warm), ds, lens, n, rets)
                    L.hvws_feeder_flush(feeder)
                else:
                    L.hvws_wsp_feed_many((ctypes.c_void_p * n)(*warm), ds, lens, n, rets)
                for h in warm:
                    L.hvws_wsp_free(h)
                t0 = time.perf_counter()
                for it in range(iters):
                    ds_np[:] = base + np.uint64(it * step)
                    if feeder:
                        L.hvws_wsp_feeder_submit(feeder, hv, ds, lens, n, rets)
                    elif mode.startswith("gpu_many"):
                        L.hvws_wsp_feed_many(hv, ds, lens, n, rets)
                    else:
                        for i in range(n):
                            L.hvws_wsp_feed(hs[i], ds[i], READ)
                if feeder:
                    L.hvws_feeder_flush(feeder)
                dt = time.perf_counter() - t0
                if feeder:
                    L.hvws_feeder_free(feeder)
            if arena:
                bufs = None
                L.hvws_host_free(eng.ctx, arena)
                for h in hs:
                    L.hvws_wsp_free(h)
            res[mode] = {
                "iteration_us": round(dt / iters * 1e6, 1),
                "GiBps_payload": round(n * iters * payload_per_read / dt / 2**30, 3),
            }
        res["cpu_kind"] = kind
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
