#!/usr/bin/env python3
"""bench.py -- device-resident WebSocket receive (header parse + unmask) on MI355X.

One step = one pass of the hot path over one synthetic batch already resident
in HBM: k_scan (frame discovery + FIN/opcode/mask/length parse) + k_unmask
(in-place rotating-key XOR), through the C ABI of libhv_amd/libhvws.so.
Default workload: BASELINE.json configs[2] (1M x 64 KiB masked binary frames,
68.7 GB on one GPU), delivered as --segments connections in one contiguous
rx buffer.  N GPUs: one process per GPU, disjoint batches (distinct seeds),
no collectives on the data path (weak scaling); gloo carries only the
barrier and the max-over-ranks time.

Also reported (not `value`): a STREAM-style in-place ceiling on the same
buffer, the host-memory-inclusive rate (pinned H2D -> scan -> unmask -> D2H,
hvws_pipeline), and the reference CPU path (oracle/_ref: libhv's own
websocket_parser.c driven through a restatement of WebSocketParser.cpp,
8 KiB chunks) timed on this host on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)

CONFIGS = {
    "c2": ("1M x 1 KiB masked binary frames (BASELINE configs[1])", "c2"),
    "c3": ("1M x 64 KiB masked binary frames (BASELINE configs[2])", "c3"),
    "c4": ("mixed 128 B-1 MiB masked frames incl. FIN=0 fragments, ~4 GiB (BASELINE configs[3])", "c4"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--segments", type=int, default=4096,
                    help="connections the batch is cut into (1 = one stream)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="budget for the CPU baseline (0: skip)")
    ap.add_argument("--cpu-sample-mib", type=int, default=256)
    ap.add_argument("--host-gib", type=float, default=4.0, help="host-inclusive sample size (0: skip)")
    ap.add_argument("--host-chunk-mib", type=int, default=64, help="hvws_pipeline chunk size")
    ap.add_argument("--sweep-unmask", action="store_true",
                    help="rank 0: time every k_unmask geometry on the same batch (design record)")
    ap.add_argument("--no-tx", action="store_true", help="skip the transmit-side (hvws_build_frames) measurement")
    ap.add_argument("--validate", action="store_true",
                    help="RFC 6455 header validation on (hvws_set_validation, all classes; off = reference behaviour)")
    ap.add_argument("--feed-conns", type=int, default=1024,
                    help="event-loop leg: connections per poll iteration (0: skip)")
    ap.add_argument("--feed-iters", type=int, default=20, help="event-loop leg: poll iterations (8 KiB reads each)")
    ap.add_argument("--dropin-reads", type=int, default=2000,
                    help="drop-in leg: FeedRecvData calls per pass, one 8 KiB read each, resident worker "
                         "against a launch per call (0: skip; scripts/bench_dropin.py runs it alone)")
    ap.add_argument("--serial", action="store_true",
                    help="hvws_step (discovery after the previous unmask) instead of hvws_step_resident")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the rank launcher and the timing reductions: no GPU call, "
                         "no measurement (tests/test_distributed.py)")
    return ap.parse_args()


def visible_devices() -> int:
    """GPUs this process could use, counted without initialising any of them
    (the launcher parent makes no GPU call): HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES when set, else the KFD topology's GPU nodes."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip()])
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for node in os.listdir(base):
            try:
                props = open(os.path.join(base, node, "properties")).read().split("\n")
            except OSError:
                continue
            simd = [ln.split()[1] for ln in props if ln.startswith("simd_count ")]
            if simd and int(simd[0]) > 0:
                n += 1
    except OSError:
        pass
    return n


def launch_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: one child
    process per GPU, as libhv runs one event loop per worker thread
    (http/server/HttpServer.cpp:216-233) and as `torch.distributed.run` would
    start them -- RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in each child's
    environment, rendezvous on 127.0.0.1.  This process makes no GPU call.
    Rank 0's JSON line is relayed to stdout; the exit status is non-zero when
    any rank fails (the others are then stopped).  Fewer visible GPUs than N
    is an error, except under HVWS_BENCH_DEVICE (every rank on one card, a
    rehearsal) or --dry-run."""
    import signal
    import socket
    import subprocess

    n = args.gpus
    rehearsal = "HVWS_BENCH_DEVICE" in os.environ or args.dry_run
    if not rehearsal:
        have = visible_devices()
        if have < n:
            print(f"bench.py: --gpus {n} but {have} GPU(s) visible; refusing to run fewer ranks "
                  "(HVWS_BENCH_DEVICE=<d> rehearses N ranks on one card)", file=sys.stderr, flush=True)
            return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    # a launcher stopped by a signal (the driver's timeout) stops its ranks
    # too: they run in sessions of their own and would keep their GPUs
    def forward(signum, _frame):
        stop_all(signum)
        raise SystemExit(128 + signum)

    old_handlers = {sg: signal.signal(sg, forward) for sg in (signal.SIGTERM, signal.SIGINT)}
    limit = float(os.environ.get("HVWS_BENCH_RANK_TIMEOUT", "0") or 0)   # seconds, 0 = none
    t_start = time.monotonic()
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                          stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                          start_new_session=True))
        chunks = []   # rank 0's stdout, read beside the polling loop (a failed rank must not wait on it)
        reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read().decode()), daemon=True)
        reader.start()
        rcs = [None] * n
        failed = False
        while any(rc is None for rc in rcs):
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    rcs[r] = p.poll()
                    if rcs[r] not in (None, 0):
                        failed = True
            if limit and time.monotonic() - t_start > limit:
                print(f"bench.py: ranks still running after {limit:.0f} s (HVWS_BENCH_RANK_TIMEOUT)",
                      file=sys.stderr, flush=True)
                failed = True
            if failed:
                break
            time.sleep(0.05)
        if failed:
            stop_all()
            for r, p in enumerate(procs):
                try:
                    rcs[r] = p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
                    rcs[r] = p.wait()
            print(f"bench.py: rank exit codes {rcs}", file=sys.stderr, flush=True)
            return 1
        reader.join(timeout=30)
    finally:
        stop_all(signal.SIGKILL)
        for sg, h in old_handlers.items():
            signal.signal(sg, h)
    line = [ln for ln in "".join(chunks).splitlines() if ln.startswith("{")]
    if not line:
        print("bench.py: rank 0 printed no result line", file=sys.stderr, flush=True)
        return 1
    # the line must name N distinct cards (outside a rehearsal)
    try:
        buses = [r.get("pci_bus_id") for r in json.loads(line[-1]).get("timing", {}).get("per_rank", [])]
    except ValueError:
        buses = []
    if len(buses) != n or ("HVWS_BENCH_DEVICE" not in os.environ and len(set(buses)) != n):
        print(f"bench.py: rank 0's line names devices {buses} for {n} ranks", file=sys.stderr, flush=True)
        return 1
    print(line[-1], flush=True)
    return 0


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(sample: np.ndarray, seconds: float, threads: int):
    """Reference CPU path on `sample` (whole frames): WebSocketParser semantics
    fed in 8 KiB chunks (event/hevent.h:16).  Each pass re-XORs the payload,
    which is the same work.  Returns (GiB/s of payload, kind, passes)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import wsharness as H

    if H.have_ref():
        L, kind = H.ref(), "reference"
    else:
        L, kind = H.oracle(), "port"
    out = (ctypes.c_uint64 * 4)()
    bufs = [sample.copy() for _ in range(threads)]
    # one pass to learn the payload bytes per pass
    rc = L.msgp_bench_feed(bufs[0].ctypes.data, bufs[0].nbytes, 8192, out)
    assert rc == 0
    payload = int(out[1])
    t0 = time.perf_counter()
    L.msgp_bench_feed(bufs[0].ctypes.data, bufs[0].nbytes, 8192, out)
    one = max(time.perf_counter() - t0, 1e-6)
    passes = max(1, int(seconds / one))
    counts = [0] * threads

    def work(i):
        o = (ctypes.c_uint64 * 4)()
        for _ in range(passes):
            L.msgp_bench_feed(bufs[i].ctypes.data, bufs[i].nbytes, 8192, o)
            counts[i] += 1

    t0 = time.perf_counter()
    ths = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    return payload * sum(counts) / dt / 2**30, kind, passes, payload * sum(counts)


def cpu_decode_only(sample: np.ndarray, plan, seconds: float):
    """Reference websocket_decode alone (http/websocket_parser.c:182-189) over
    the masked payload spans of the sample's frames, one core: the XOR the
    GPU kernel replaces, without parsing or message assembly."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import wsharness as H
    from libhv_amd import synth

    L = H.ref() if H.have_ref() else H.oracle()
    hdr = synth.frame_size(plan.flags, plan.length) - plan.length
    end = plan.frame_off + synth.frame_size(plan.flags, plan.length)
    m = int(np.searchsorted(end, sample.nbytes, side="right"))
    sel = (plan.flags[:m] & synth.MASK) != 0
    off = np.ascontiguousarray((plan.frame_off[:m] + hdr[:m])[sel], dtype=np.uint64)
    ln = np.ascontiguousarray(plan.length[:m][sel], dtype=np.uint64)
    key = np.ascontiguousarray(plan.mask[:m][sel], dtype=np.uint32)
    buf = sample.copy()
    L.msgp_bench_decode_spans.restype = ctypes.c_uint64
    L.msgp_bench_decode_spans.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t]
    args = (buf.ctypes.data, off.ctypes.data, ln.ctypes.data, key.ctypes.data, len(ln))
    t0 = time.perf_counter()
    per = L.msgp_bench_decode_spans(*args)
    one = max(time.perf_counter() - t0, 1e-6)
    passes = max(1, int(seconds / one))
    t0 = time.perf_counter()
    for _ in range(passes):
        L.msgp_bench_decode_spans(*args)
    dt = time.perf_counter() - t0
    return per * passes / dt / 2**30


def pcie_ceiling(device: int, nbytes: int = 1 << 30, piece: int = 64 << 20, reps: int = 3) -> dict:
    """This box's host link, measured in the same run with the HIP runtime
    directly and the same call pattern as hvws_pipeline (pinned buffers,
    `piece`-sized hipMemcpyAsync on non-blocking streams): H2D alone, D2H
    alone, and both at once on two streams.  GB/s per direction."""
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    hip.hipSetDevice(device)
    h_in, h_out, d_in, d_out, s1, s2 = vp(), vp(), vp(), vp(), vp(), vp()
    assert hip.hipHostMalloc(ctypes.byref(h_in), ctypes.c_size_t(nbytes), 0) == 0
    assert hip.hipHostMalloc(ctypes.byref(h_out), ctypes.c_size_t(nbytes), 0) == 0
    assert hip.hipMalloc(ctypes.byref(d_in), ctypes.c_size_t(nbytes)) == 0
    assert hip.hipMalloc(ctypes.byref(d_out), ctypes.c_size_t(nbytes)) == 0
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s1), 1) == 0   # hipStreamNonBlocking
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s2), 1) == 0
    H2D, D2H = 1, 2   # hipMemcpyHostToDevice, hipMemcpyDeviceToHost

    def run(h2d: bool, d2h: bool) -> float:
        best = None
        for _ in range(reps):
            hip.hipDeviceSynchronize()
            t = time.perf_counter()
            for o in range(0, nbytes, piece):
                n = ctypes.c_size_t(min(piece, nbytes - o))
                if h2d:
                    hip.hipMemcpyAsync(vp(d_in.value + o), vp(h_in.value + o), n, H2D, s1)
                if d2h:
                    hip.hipMemcpyAsync(vp(h_out.value + o), vp(d_out.value + o), n, D2H, s2)
            hip.hipStreamSynchronize(s1)
            hip.hipStreamSynchronize(s2)
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        return best

    t_in, t_out, t_both = run(True, False), run(False, True), run(True, True)
    for p in (d_in, d_out):
        hip.hipFree(p)
    for p in (h_in, h_out):
        hip.hipHostFree(p)
    hip.hipStreamDestroy(s1)
    hip.hipStreamDestroy(s2)
    return {"h2d_GBps": round(nbytes / t_in / 1e9, 2), "d2h_GBps": round(nbytes / t_out / 1e9, 2),
            "concurrent_GBps_per_direction": round(nbytes / t_both / 1e9, 2), "bytes": nbytes, "piece": piece}


FEED_READ = 8192   # event/hevent.h:16 HLOOP_READ_BUFSIZE


def event_loop_leg(eng, device: int, conns: int, iters: int, seed: int):
    """SURVEY 8(f) row 1 inside the run: `conns` connections each deliver
    `iters` 8 KiB reads of a stream of masked 1 KiB binary frames (device
    synth); one poll iteration hands every connection's next read over.
    Read buffers are one pinned arena (hvws_host_alloc), a poll iteration's
    reads side by side, so the reads go to the kernel in place (hvws_rx_reads).
    Timed: hvws_feeder_submit per iteration + the final flush (pipelined), and
    hvws_wsp_feed_many per iteration (synchronous), each over a whole pass with
    fresh parsers: the median of 3 passes each, after one untimed pass of each.  Returns (result dict, the masked
    streams for the CPU reference, their payload bytes)."""
    import libhv_amd
    from libhv_amd import synth

    L = libhv_amd.lib()
    L.hvws_set_thread_device(device)
    per = FEED_READ * iters
    fp = synth.uniform_plan(conns * (per // 1032 + 2), 1024, seed).split(conns)
    dpf = libhv_amd.DevicePlan(eng, fp)
    buf = eng.alloc(fp.total + 64)
    eng.synth(buf, fp.total, fp.seed, dpf, 0)
    host = buf.download(fp.total)
    buf.free()
    dpf.free()
    streams = np.stack([host[o:o + per] for o, _ in fp.segments])   # (conns, per), masked
    arena = L.hvws_host_alloc(eng.ctx, conns * per)
    ring = np.ctypeslib.as_array((ctypes.c_uint8 * (conns * per)).from_address(arena))
    ring.reshape(iters, conns, FEED_READ)[:] = streams.reshape(conns, iters, FEED_READ).transpose(1, 0, 2)
    lens = (ctypes.c_size_t * conns)(*([FEED_READ] * conns))
    rets = (ctypes.c_int * conns)()
    ds = (ctypes.c_void_p * conns)()
    ds_np = np.frombuffer(ds, dtype=np.uint64)
    base = np.uint64(arena) + np.arange(conns, dtype=np.uint64) * np.uint64(FEED_READ)

    feeder = L.hvws_feeder_new()   # one feeder (its worker context stays warm across passes)

    def one_pass(pipelined: bool) -> float:
        hs = [L.hvws_wsp_new() for _ in range(conns)]
        hv = (ctypes.c_void_p * conns)(*hs)
        t = time.perf_counter()
        for it in range(iters):
            ds_np[:] = base + np.uint64(it * conns * FEED_READ)
            if pipelined:
                L.hvws_wsp_feeder_submit(feeder, hv, ds, lens, conns, rets)
            else:
                L.hvws_wsp_feed_many(hv, ds, lens, conns, rets)
        if pipelined:
            L.hvws_feeder_flush(feeder)
        dt = time.perf_counter() - t
        for h in hs:
            L.hvws_wsp_free(h)
        assert all(r == FEED_READ for r in rets), "event-loop leg: a read was not consumed"
        return dt

    # each pass unmasks (or re-masks) every read in place: the same work;
    # one untimed pass per mode first (contexts, staging, first launches),
    # then the median of 3 timed passes of each, interleaved
    one_pass(True)
    one_pass(False)
    tp, ts = [], []
    for _ in range(3):
        tp.append(one_pass(True))
        ts.append(one_pass(False))
    t_pipe, t_sync = float(np.median(tp)), float(np.median(ts))
    L.hvws_feeder_free(feeder)
    L.hvws_host_free(eng.ctx, arena)
    pay = conns * iters * FEED_READ * 1024 / 1032
    res = {
        "connections": conns, "read_bytes": FEED_READ, "iterations": iters, "frames": "masked 1 KiB binary",
        "pipelined_us_per_iteration": round(t_pipe / iters * 1e6, 1),
        "GiBps_payload": round(pay / t_pipe / 2**30, 3),
        "batched_us_per_iteration": round(t_sync / iters * 1e6, 1),
        "batched_GiBps_payload": round(pay / t_sync / 2**30, 3),
        "api": "hvws_feeder_submit (pipelined) / hvws_feed_many over hvws_host_alloc read buffers (hvws_rx_reads)",
    }
    return res, streams, pay


def dropin_leg(eng, device: int, seed: int, reads: int = 2000, builds: int = 4000, passes: int = 3) -> dict:
    """The literal drop-in's per-call latency (SURVEY 8(f) row 1 as libhv calls
    it unchanged): WebSocketParser::FeedRecvData once per 8 KiB read
    (http/server/HttpHandler.cpp:757-763) on one connection, and a masked
    125-byte websocket_build_frame per message (http/WebSocketChannel.cpp:66-79
    via ws_build_frame).  Timed in C (tests/csrc/callbench.c), no interpreter
    in the loop; the resident worker (hvws_set_door) on and off, interleaved,
    median of `passes`; the reference on one core beside it."""
    import libhv_amd
    from libhv_amd import synth

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import wsharness as H

    L = libhv_amd.lib()
    L.hvws_set_thread_device(device)
    CB = ctypes.CDLL(os.path.join(ROOT, "tests", "_build", "libcallbench.so"))
    CB.cb_feed.restype = ctypes.c_double
    CB.cb_feed.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t] * 2
    CB.cb_build.restype = ctypes.c_double
    CB.cb_build.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_size_t, ctypes.c_int]
    total = FEED_READ * reads
    fp = synth.uniform_plan(total // 1032 + 2, 1024, seed)
    dpf = libhv_amd.DevicePlan(eng, fp)
    buf = eng.alloc(fp.total + 64)
    eng.synth(buf, fp.total, fp.seed, dpf, 0)
    masked = buf.download(fp.total)[:total].copy()
    buf.free()
    dpf.free()
    work = np.empty_like(masked)
    R = H.ref() if H.have_ref() else H.oracle()
    addr = lambda lib, f: ctypes.cast(getattr(lib, f), ctypes.c_void_p).value  # noqa: E731

    def feed_once(impl: str) -> float:
        work[:] = masked
        if impl == "ref":
            h = R.msgp_new()
            dt = CB.cb_feed(addr(R, "msgp_feed"), h, work.ctypes.data, total, FEED_READ)
            R.msgp_free(h)
        else:
            L.hvws_set_door(None, 1 if impl == "door" else 0)
            h = L.hvws_wsp_new()
            dt = CB.cb_feed(addr(L, "hvws_wsp_feed"), h, work.ctypes.data, total, FEED_READ)
            L.hvws_wsp_free(h)
        assert dt > 0, f"drop-in leg: a read was not consumed ({impl})"
        return dt / reads * 1e6

    payload = np.frombuffer(np.random.default_rng(seed).bytes(125), np.uint8).copy()
    key = ctypes.create_string_buffer(b"\x12\x34\x56\x78", 4)
    out = ctypes.create_string_buffer(256)

    def build_once(impl: str) -> float:
        if impl == "ref":
            fn = addr(R, "websocket_build_frame" if H.have_ref() else "ows_build_frame")
        else:
            L.hvws_set_door(None, 1 if impl == "door" else 0)
            fn = addr(L, "websocket_build_frame")
        dt = CB.cb_build(fn, out, 0x2 | 0x10 | 0x20, key, payload.ctypes.data, 125, builds)
        assert dt > 0, f"drop-in leg: build_frame size mismatch ({impl})"
        return dt / builds * 1e6

    for impl in ("door", "launch", "ref"):   # warm: worker resident, contexts and buffers made
        feed_once(impl)
        build_once(impl)
    res = {k: [] for k in ("feed_door", "feed_launch", "feed_ref", "build_door", "build_launch", "build_ref")}
    for _ in range(passes):
        for impl in ("door", "launch", "ref"):
            res["feed_" + impl].append(feed_once(impl))
            res["build_" + impl].append(build_once(impl))
    L.hvws_set_door(None, 0)    # the worker parks now, not after its idle time
    L.hvws_set_door(None, -1)   # the default again (on), nothing resident
    # the leg's thread context goes now, worker and its CU-masked stream with
    # it (a process under rocprofv3 that still held such a stream at exit
    # crashed in its exit-time destructors, profiles/r3x_rocprof_c3.md)
    L.hvws_thread_release()
    med = {k: round(float(np.median(v)), 2) for k, v in res.items()}
    return {
        "feed_8KiB_read_us": {"resident_worker": med["feed_door"], "launch_per_call": med["feed_launch"],
                              "reference_1core": med["feed_ref"]},
        "build_frame_125B_masked_us": {"resident_worker": med["build_door"], "launch_per_call": med["build_launch"],
                                       "reference_1core": med["build_ref"]},
        "reads": reads, "builds": builds,
        "note": "WebSocketParser::FeedRecvData per 8 KiB read of 1 KiB masked frames (pageable buffer, one "
                "connection) and masked websocket_build_frame of 125 B, per call, timed in C; median of "
                f"{passes} interleaved passes",
    }


def dropin_leg_child(device: int, seed: int, reads: int) -> dict:
    """dropin_leg in a child process of its own (scripts/bench_dropin.py), as a
    libhv server process would call the drop-in: in this process -- after the
    workload legs, with torch and the rank's other contexts loaded -- the same
    calls measured ~0.7 us slower each (builds 4.1-4.2 vs 3.4-3.8 us on one
    box, profiles/r5_raw/door).  A child is started, not exec'd."""
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "bench_dropin.py"), str(reads), str(device), str(seed)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        raise SystemExit(f"drop-in leg: child exited {r.returncode}: {r.stderr[-2000:]}")
    res = json.loads(lines[-1])
    res["process"] = "a child process of its own (scripts/bench_dropin.py), like a libhv server process"
    return res


def cpu_event_loop(streams: np.ndarray, iters: int, pay: float):
    """The reference parser + WebSocketParser message layer on one core over
    the same reads, connection by connection per poll iteration."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import wsharness as H

    R = H.ref() if H.have_ref() else H.oracle()
    bufs = np.array(streams, copy=True)
    conns = bufs.shape[0]
    hs = [R.msgp_new() for _ in range(conns)]
    addr = [bufs[i].ctypes.data for i in range(conns)]
    t = time.perf_counter()
    for it in range(iters):
        for i in range(conns):
            R.msgp_feed(hs[i], addr[i] + it * FEED_READ, FEED_READ)
    dt = time.perf_counter() - t
    for h in hs:
        R.msgp_free(h)
    return {"us_per_iteration": round(dt / iters * 1e6, 1), "GiBps_payload": round(pay / dt / 2**30, 3), "cores": 1}


def cpu_info() -> dict:
    """CPU model and the CPUs this process may use: nproc (affinity) and the
    cgroup's CPU quota (cpu.max), whichever is smaller."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    usable = min(nproc, quota) if quota else nproc
    return {"cpu_model": model, "nproc": nproc, "cgroup_cpus": quota, "usable_cpus": usable}


def gather_rows(dist, row) -> np.ndarray:
    """Every rank's `row` (floats), as a (world, len(row)) array on every rank
    (gloo all_gather; a single row when not distributed).  Timing only -- no
    data-path collective."""
    r = np.asarray(row, dtype=np.float64)
    if dist is None:
        return r[None, :]
    import torch

    t = torch.tensor(r)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return np.stack([o.numpy() for o in out])


def span_of(rows: np.ndarray, i_start: int = 0, i_end: int = 1) -> float:
    """max over ranks of end - min over ranks of start (one host clock:
    time.perf_counter is CLOCK_MONOTONIC, shared by the processes of a node)."""
    return float(rows[:, i_end].max() - rows[:, i_start].min())


def init_dist():
    """(rank, world, local_rank, dist-or-None).  One process per GPU; gloo
    carries only the barrier and the timing reduction (no data collectives)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo's C++ side prints its connection messages to stdout; the one
        # JSON line must be alone there, so fd 1 points at stderr meanwhile
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return rank, world, local, dist


def rank_seed(cfg: str, rank: int) -> int:
    """This rank's batch seed: c3 ranks take config 5's shards (seed 1000 + r,
    fixtures c5_rank<r>); c1 / c2 / c4 ranks take seed 1 + r, so rank 0's batch
    is the one tests/golden/configs.json holds the reference digests of."""
    return 1000 + rank if cfg == "c3" else 1 + rank


def rank_plan(cfg: str, rank: int, segments: int):
    """This rank's disjoint batch: same shape on every rank, distinct seed."""
    from libhv_amd import synth

    return synth.config_plan(cfg, seed=rank_seed(cfg, rank)).split(segments)


def max_over_ranks(dist, seconds: float) -> float:
    if dist is None:
        return seconds
    import torch

    t = torch.tensor([seconds], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_inclusive_leg(eng, plan, dp, rx, args, dist, rank: int, world: int, device: int):
    """Host memory in, host memory out: the first ~host_gib of
    this rank's batch from pinned host memory through hvws_pipeline (chunked
    H2D -> scan -> unmask -> D2H, 3-slot ring).  Every rank runs it at the
    same time -- each call starts after a gloo barrier -- so with N GPUs the
    links and host DRAM are shared as in a real N-GPU server (SURVEY sec. 7
    hard part 4).  Returns (this rank's row, rank-0-only result or None,
    the CPU sample (rank 0) or None)."""
    import libhv_amd
    from libhv_amd import synth

    L = libhv_amd.lib()
    sizes = synth.frame_size(plan.flags, plan.length)
    ends = np.cumsum(sizes)
    m = int(np.searchsorted(ends, int(args.host_gib * 2**30), side="right"))
    m = max(1, min(m, plan.n))
    hbytes = int(ends[m - 1])
    pay = float(plan.length[:m].sum())
    eng.synth(rx, plan.total, plan.seed, dp, 0)
    pinned = L.hvws_host_alloc(eng.ctx, hbytes)
    host = np.ctypeslib.as_array((ctypes.c_uint8 * hbytes).from_address(pinned))
    libhv_amd._check(L.hvws_d2h(eng.ctx, pinned, rx.ptr, hbytes), "d2h")
    eng.sync()
    sample = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        # CPU baseline sample = the first whole frames of the same (masked) batch
        ms = max(1, int(np.searchsorted(ends, args.cpu_sample_mib << 20, side="right")))
        sample = np.array(host[: int(ends[ms - 1])], copy=True)
    chunk = args.host_chunk_mib << 20
    # one untimed call (slot allocation, the link warming up), then 3 timed
    # calls, all ranks starting each call together; each call toggles the
    # host bytes between masked and unmasked
    rows = []
    for r in range(4):
        carry = libhv_amd.WsParser()
        L.websocket_parser_init(ctypes.byref(carry))
        if dist is not None:
            dist.barrier()
        t = time.perf_counter()
        libhv_amd._check(L.hvws_pipeline(eng.ctx, pinned, hbytes, chunk, ctypes.byref(carry)), "pipeline")
        t1 = time.perf_counter()
        if r:
            rows.append(gather_rows(dist, [t, t1, hbytes, pay]))
    L.hvws_host_free(eng.ctx, pinned)
    if dist is not None:
        dist.barrier()
    link = pcie_ceiling(device, piece=chunk)   # every rank at once, like the pipeline
    lrows = gather_rows(dist, [link["h2d_GBps"], link["d2h_GBps"], link["concurrent_GBps_per_direction"]])
    if rank != 0:
        return None, sample
    # per call: the aggregate over ranks = all bytes / (latest end - earliest start)
    agg = [float(x[:, 2].sum()) / span_of(x) for x in rows]
    agg_pay = [float(x[:, 3].sum()) / span_of(x) for x in rows]
    k = int(np.argsort(agg)[len(agg) // 2])   # median call
    per_rank = []
    for q in range(rows[0].shape[0]):
        dts = [float(x[q, 1] - x[q, 0]) for x in rows]
        dt = float(np.median(dts))
        per_rank.append({"rank": q, "GBps_wire": round(hbytes / dt / 1e9, 2),
                         "GiBps_payload": round(pay / dt / 2**30, 2),
                         "link_concurrent_GBps_per_direction": float(lrows[q, 2]),
                         "frac_of_own_link": round(hbytes / dt / 1e9 / float(lrows[q, 2]), 3)})
    link_sum = float(lrows[:, 2].sum())
    res = {
        "GiBps_payload": per_rank[0]["GiBps_payload"],
        "GBps_wire": per_rank[0]["GBps_wire"],
        "frac_of_concurrent_link": per_rank[0]["frac_of_own_link"],
        "bytes": hbytes, "chunk": chunk,
        "note": "pinned H2D + scan + unmask + D2H, 3-slot ring, PCIe-bound; median of 3 calls after 1 warm-up; "
                "all ranks run each call together (gloo barrier before each)",
        "link": link,
        "per_rank": per_rank,
        "aggregate": {
            "GBps_wire": round(agg[k] / 1e9, 2),
            "GiBps_payload": round(agg_pay[k] / 2**30, 2),
            "ranks": world,
            "sum_of_links_GBps_per_direction": round(link_sum, 2),
            "frac_of_sum_of_links": round(agg[k] / 1e9 / link_sum, 3),
            "method": "all ranks' bytes / (latest end - earliest start) per call, host CLOCK_MONOTONIC; "
                      "median call of 3; links measured concurrently on every rank",
        },
    }
    return res, sample


def tx_leg(eng, plan, dp, rx, rx_plain: bool, segs, tpath: str) -> dict:
    """Transmit side: rebuild every frame of the batch
    from its plaintext payload with hvws_build_frames; the output must be the
    masked batch byte for byte."""
    import libhv_amd
    from libhv_amd import synth

    if not rx_plain:
        eng.step(rx, plan.total, segs)   # leave rx holding plaintext payloads
    hdr = synth.frame_size(plan.flags, plan.length) - plan.length
    tx = libhv_amd.TxPlan(eng, plan.frame_off + hdr, plan.length, plan.flags, plan.mask)
    out_buf = eng.alloc(plan.total + 64)
    tms = []
    for _ in range(4):
        eng.build_frames(out_buf, plan.total + 64, rx, plan.total, tx)
        tms.append(eng.last_kernel_ms())
    ok = eng.synth(out_buf, plan.total, plan.seed, dp, 1) == 0
    tx_alg = plan.payload_bytes + plan.total
    tx_ach = tx_alg / (float(np.mean(tms[1:])) * 1e-3) / 1e9
    bname = libhv_amd.lib().hvws_last_build_kernel(eng.ctx).decode()
    tx_traffic = None
    if os.path.exists(tpath):
        ent = json.load(open(tpath)).get(bname, {}).get(str(plan.total))
        tx_traffic = ent["hbm_bytes"] if ent else None
    out_buf.free()
    tx.free()
    if not ok:
        raise SystemExit("transmit build differs from the masked batch")
    return {
        "kernel": bname, "traffic": tx_traffic,
        "achieved": round(tx_ach, 1), "unit": "GB/s", "frac": round(tx_ach / HBM_PEAK_GBS, 4),
        "alg_bytes_per_launch": tx_alg, "kernel_ms_mean": round(float(np.mean(tms[1:])), 3),
        "timed": "tile index + source spans + k_build (the call's device work after its size check)",
        "verified": ok,
    }


def bus_number(bus_id: str) -> int:
    """PCI bus id "dddd:bb:dd.f" as one integer (gathered over gloo as a float)."""
    dom, bus, df = bus_id.split(":")
    dv, fn = df.split(".")
    return (int(dom, 16) << 16) | (int(bus, 16) << 8) | (int(dv, 16) << 3) | int(fn, 16)


def bus_name(n: int) -> str:
    return f"{n >> 16:04x}:{(n >> 8) & 0xFF:02x}:{(n >> 3) & 0x1F:02x}.{n & 7:x}"


def check_distinct_devices(bus_ids, rank: int) -> None:
    """An N-rank line must come from N cards: two ranks on one PCI bus id
    end the run (exit status 3), except in a rehearsal (HVWS_BENCH_DEVICE
    pins every rank to one card on purpose)."""
    if "HVWS_BENCH_DEVICE" in os.environ or len(set(bus_ids)) == len(bus_ids):
        return
    print(f"bench.py: rank {rank}: ranks share a device: {bus_ids}", file=sys.stderr, flush=True)
    raise SystemExit(3)


def fixture_for(cfg: str, rank: int):
    """(name, entry) of the committed reference digests for this rank's batch,
    streamed through the reference by make_golden.py --big
    (tests/golden/configs.json): c5_rank<r> = the c3-shaped batch of seed
    1000 + r; c1 / c2 / c4 = that config's batch of seed 1 (rank 0's)."""
    path = os.path.join(ROOT, "tests", "golden", "configs.json")
    if not os.path.exists(path):
        return None, None
    name = f"c5_rank{rank}" if cfg == "c3" else (cfg if rank == 0 else None)
    if name is None:
        return None, None
    ent = json.load(open(path)).get(name)
    if ent is not None and cfg != "c3" and f"seed={rank_seed(cfg, rank)})" not in ent["plan"]["fn"]:
        return None, None
    return name, ent


def start_watchdog(period: float) -> None:
    """A run still going after `period` seconds (and every `period` after)
    leaves its state on stderr: every thread's Python stack, every thread's
    native stack (hvws_debug_backtraces) and the library's contexts -- each
    resident worker's mailbox and every stream's hipStreamQuery
    (hvws_debug_dump, memory state first).  Diagnostics only ($HVWS_BENCH_WATCHDOG
    seconds, 0: off)."""
    import faulthandler

    def run():
        n = 0
        while True:
            time.sleep(period)
            n += 1
            print(f"[bench] watchdog: still running after {n * period:.0f} s", file=sys.stderr, flush=True)
            faulthandler.dump_traceback(all_threads=True)
            try:
                import libhv_amd

                L = libhv_amd.lib()
                print(f"[bench] native stacks ({L.hvws_debug_backtraces(2)} threads answered above)",
                      file=sys.stderr, flush=True)
                L.hvws_debug_dump(2)
            except Exception as e:   # noqa: BLE001 -- diagnostics must not end the run
                print(f"[bench] watchdog: {e!r}", file=sys.stderr, flush=True)

    threading.Thread(target=run, name="bench-watchdog", daemon=True).start()


def per_rank_roofline(row) -> dict:
    """One rank's own unmask time, its fraction of 8 TB/s and of its card's
    in-place ceiling (row = [unmask ms mean, achieved GB/s, ceiling GB/s])."""
    ms, achieved, ceiling = (float(x) for x in row)
    return {"unmask_ms_mean": round(ms, 3),
            "roofline_frac": round(achieved / HBM_PEAK_GBS, 4),
            "stream_ceiling_GBps": round(ceiling, 1),
            "frac_of_box_ceiling": round(achieved / ceiling, 4) if ceiling > 0 else None}


def dry_run(args, rank: int, world: int, local: int, dist) -> None:
    """--dry-run: the rank plumbing of a real run with the GPU legs stubbed --
    every rank builds its disjoint batch plan (CPU), the timing rows and the
    digest-fixture mapping go through the same gloo reductions, rank 0 prints
    the same keys.  No GPU call, no measurement."""
    plan = rank_plan("c1", rank, 8)
    if os.environ.get("HVWS_BENCH_DRYRUN_FAIL_RANK") == str(rank):
        raise SystemExit(f"rank {rank}: failing on request (HVWS_BENCH_DRYRUN_FAIL_RANK)")
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    t1 = time.perf_counter()
    # no device: a stand-in bus id per local rank ($HVWS_BENCH_DRYRUN_BUS pins
    # every rank to one, as two ranks on one card would report)
    bus = os.environ.get("HVWS_BENCH_DRYRUN_BUS", f"0000:{local + 1:02x}:00.0")
    trows = gather_rows(dist, [t0, t1, 0.0, local, local, bus_number(bus)])
    check_distinct_devices([bus_name(int(b)) for b in trows[:, 5]], rank)
    fx_name, fx = fixture_for("c3", rank)
    vrows = gather_rows(dist, [rank, local, int(plan.seed), -1 if fx is None else 1])
    # stand-in per-rank unmask times and ceilings ($HVWS_BENCH_DRYRUN_SLOW_RANK
    # makes one rank's card slow), through the same gather as a real run
    slow = os.environ.get("HVWS_BENCH_DRYRUN_SLOW_RANK") == str(rank)
    ms = 21.3 * (1.5 if slow else 1.0)
    prows = gather_rows(dist, [ms, 137.4536e9 / (ms * 1e-3) / 1e9, 6460.0])
    if rank == 0:
        print(json.dumps({
            "metric": "device-resident WS unmask GiB/s, 64 KiB masked frames, 1/2/4/8 MI355X",
            "value": None, "unit": "GiB/s", "n_gpus": world, "dry_run": True,
            "timing": {"elapsed_s": span_of(trows),
                       "per_rank": [{"rank": int(r), "device": int(trows[r, 3]), "hip_device": int(trows[r, 4]),
                                     "pci_bus_id": bus_name(int(trows[r, 5])),
                                     "start_offset_ms": round(float(trows[r, 0] - trows[:, 0].min()) * 1e3, 3),
                                     **per_rank_roofline(prows[r])}
                                    for r in range(trows.shape[0])]},
            "verified": {"ranks": [{"rank": int(v[0]), "local_rank": int(v[1]), "seed": int(v[2]),
                                    "fixture": f"c5_rank{int(v[0])}" if v[3] >= 0 else None} for v in vrows]},
        }), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    wd = float(os.environ.get("HVWS_BENCH_WATCHDOG", "150") or 0)
    if wd > 0:
        start_watchdog(wd)
    rank, world, local, dist = init_dist()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        dry_run(args, rank, world, local, dist)
        return
    if world > 1:
        # The CPU baseline is taken at N = 1 only.  At N > 1 every rank runs
        # the timed steps and the host-inclusive leg (together, so links and
        # host DRAM are shared as in production); rank 0 alone runs the
        # transmit and event-loop legs.
        args.cpu_seconds = 0
    import torch

    import libhv_amd

    def barrier():
        eng.sync()
        if torch.cuda.is_available():
            torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()

    desc, cfg = CONFIGS[args.config]
    # one process per GPU: LOCAL_RANK picks the device (modulo the visible
    # count, so a launcher that narrows HIP_VISIBLE_DEVICES per rank also
    # works); HVWS_BENCH_DEVICE pins every rank to one card for rehearsals.
    ndev = max(1, libhv_amd.device_count())
    device = int(os.environ.get("HVWS_BENCH_DEVICE", local % ndev))
    bus_id, hip_device = libhv_amd.device_identity(device)
    eng = libhv_amd.Engine(device)
    t = time.perf_counter()
    plan = rank_plan(cfg, rank, args.segments)
    dp = libhv_amd.DevicePlan(eng, plan)
    rx = eng.alloc(plan.total + 64)
    eng.synth(rx, plan.total, plan.seed, dp, 0)
    eng.sync()
    log(rank, f"[bench] {plan.n} frames, {plan.total / 1e9:.2f} GB rx, {len(plan.segments)} segments, "
              f"built in {time.perf_counter() - t:.2f}s")
    P = plan.masked_payload_bytes()
    HB = plan.header_bytes
    segs = eng.prepare(plan.segments)   # ctypes tables built once, outside the timed loop
    fx_name, fx = fixture_for(cfg, rank)
    if fx is not None:
        # the batch this rank built is the reference's (masked digest)
        d = f"{eng.digest(rx, plan.total):016x}"
        if d != fx["digest_masked"]:
            raise SystemExit(f"rank {rank}: masked batch digest {d} != {fx_name} {fx['digest_masked']}")

    # The batch is resident in HBM before the timed region, so steps use
    # hvws_step_resident: each step's discovery (second stream) overlaps the
    # previous step's unmask; every step still scans and unmasks the whole
    # batch (the same buffer: headers are never modified, payloads toggle).
    step = eng.step if args.serial else eng.step_resident
    L = libhv_amd.lib()
    if args.validate:
        L.hvws_set_validation(eng.ctx, 0x3F)   # HVWS_V_ALL
    for _ in range(args.warmup):
        step(rx, plan.total, segs)
    barrier()
    # Steps are issued back to back (each still synchronises once inside its
    # scan to size the frame table); the per-launch kernel times are read
    # from the engine's event ring after the timed region.  Per device: span
    # markers on the context's streams (hvws_span_*); across devices: the
    # host's CLOCK_MONOTONIC (time.perf_counter), common to all ranks of the
    # node -- value = all payload / (latest end - earliest start).
    # Kernel times come from HIP events on sampled steps of the timed region:
    # each event-carrying step costs device time between kernels (~15 us of a
    # 0.38 ms config-2 step, profiles/r5_raw/events), so long runs carry them
    # on every 8th step only (hvws_set_step_event_interval); all launches of a
    # run are the same work.
    ev_every = 8 if args.steps >= 32 else 1
    eng.set_step_event_interval(ev_every)
    t0 = time.perf_counter()
    span_ms = ctypes.c_float(0)
    libhv_amd._check(L.hvws_span_begin(eng.ctx), "span_begin")
    for _ in range(args.steps):
        step(rx, plan.total, segs)
    libhv_amd._check(L.hvws_span_end(eng.ctx, ctypes.byref(span_ms)), "span_end")
    eng.sync()
    t1 = time.perf_counter()
    barrier()
    trows = gather_rows(dist, [t0, t1, span_ms.value, device, hip_device, bus_number(bus_id)])
    elapsed = span_of(trows)
    # every rank on its own card (a rehearsal under HVWS_BENCH_DEVICE excepted)
    check_distinct_devices([bus_name(int(b)) for b in trows[:, 5]], rank)
    scan_path = L.hvws_last_scan_path(eng.ctx)
    times = eng.step_times(min(args.steps, 32))
    eng.set_step_event_interval(1)
    scan_ms = [t[0] for t in times]
    unmask_ms = [t[1] for t in times if t[1] >= 0]   # the sampled steps
    if not unmask_ms:
        raise SystemExit(f"rank {rank}: no unmask timing events in the last {len(times)} steps")

    # The same number of steps through the other step call, for the record
    # (pipelined vs serial); an even count keeps the parity of passes.
    other_ms = None
    if rank == 0:
        other = eng.step if not args.serial else eng.step_resident
        n_other = 4
        eng.sync()
        t = time.perf_counter()
        for _ in range(n_other):
            other(rx, plan.total, segs)
        eng.sync()
        other_ms = (time.perf_counter() - t) / n_other * 1e3
    # Correctness after the timed region: an odd number of passes leaves the
    # payload unmasked, an even number masked again (XOR is an involution).
    # Byte-exact against the plan (device synth VERIFY), and -- for c3-shaped
    # batches -- the whole buffer's digest against the reference's fixture.
    passes = args.warmup + args.steps + (4 if rank == 0 else 0)
    bad = eng.synth(rx, plan.total, plan.seed, dp, 2 if passes % 2 else 1)
    if bad:
        raise SystemExit(f"rank {rank}: {bad} bytes differ from the expected batch after {passes} passes")
    digest_ok = None
    if fx is not None:
        want = fx["digest_unmasked"] if passes % 2 else fx["digest_masked"]
        d = f"{eng.digest(rx, plan.total):016x}"
        digest_ok = d == want
        if not digest_ok:
            raise SystemExit(f"rank {rank}: digest {d} after {passes} passes != reference {fx_name} {want}")
    vrows = gather_rows(dist, [rank, device, -1 if digest_ok is None else int(digest_ok)])

    value = world * plan.payload_bytes * args.steps / elapsed / 2**30
    mean_unmask = float(np.mean(unmask_ms))
    alg_bytes = 2 * P + HB
    achieved = alg_bytes / (mean_unmask * 1e-3) / 1e9

    kname = (L.hvws_run_kernel_name() if scan_path == 7 else L.hvws_unmask_kernel_name_for(plan.total)).decode()
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        ent = json.load(open(tpath)).get(kname, {}).get(str(plan.total))
        if ent:
            traffic, traffic_src = ent["hbm_bytes"], f"profiles/traffic.json ({ent['method']})"

    # Every rank: the STREAM-style in-place ceiling (read+write every byte) of
    # its own card on the same buffer (an even number of passes: no net
    # change), so an N-rank line shows each card's unmask time, its fraction
    # of 8 TB/s and of its own ceiling -- one slow card stands out.
    eng.sync()
    t = time.perf_counter()
    reps = 4
    for _ in range(reps):
        eng.stream_xor(rx, plan.total & ~15, 0x5A5A5A5A)
    eng.sync()
    ceiling = 2 * (plan.total & ~15) * reps / (time.perf_counter() - t) / 1e9
    prows = gather_rows(dist, [mean_unmask, achieved, ceiling])

    extra = {}
    sample = None
    feed_streams = feed_pay = None
    if rank == 0:
        extra["stream_ceiling_GBps"] = round(ceiling, 1)
        # pipelined steps record no scan-side timing markers (-1; include/hvws.h)
        scan_rec = [t for t in scan_ms if t >= 0]
        extra["scan_ms_mean"] = round(float(np.mean(scan_rec)), 3) if scan_rec else None
        extra["step_call"] = ("hvws_step" if args.serial else
                              "hvws_step_resident (discovery overlaps the previous unmask)")
        if args.validate:
            extra["validation"] = "HVWS_V_ALL"
        extra["other_step_call_ms"] = round(other_ms, 3) if other_ms is not None else None
        extra["scan_path"] = {0: "count_emit", 1: "count_read_emit", 2: "single", 3: "speculative",
                              4: "speculative_rejected", 5: "slack", 6: "slack_rejected", 7: "run"}.get(scan_path, scan_path)
        extra["timing"] = {
            "method": "per device: hvws_span_begin/end markers on the context's streams (HIP events); "
                      "across devices: latest end - earliest start on the host CLOCK_MONOTONIC after a barrier",
            "elapsed_s": round(elapsed, 6),
            "per_rank": [{"rank": int(r), "device": int(trows[r, 3]), "hip_device": int(trows[r, 4]),
                          "pci_bus_id": bus_name(int(trows[r, 5])),
                          "device_span_ms": round(float(trows[r, 2]), 3),
                          "start_offset_ms": round(float(trows[r, 0] - trows[:, 0].min()) * 1e3, 3),
                          "end_offset_ms": round(float(trows[r, 1] - trows[:, 0].min()) * 1e3, 3),
                          **per_rank_roofline(prows[r])}
                         for r in range(trows.shape[0])],
            "device_span_ms_max": round(float(trows[:, 2].max()), 3),
        }
        extra["verified"] = {
            "method": "every payload byte vs its plaintext (device synth VERIFY) after the run; digest of the "
                      "whole rx buffer vs the reference's (tests/golden/configs.json: c5_rank<r> for c3, the "
                      "config's own entry for rank 0 of c1/c2/c4) before and after",
            "ranks": [{"rank": int(v[0]), "device": int(v[1]),
                       "fixture": (fixture_for(cfg, int(v[0]))[0] if v[2] >= 0 else None),
                       "digest_match": (bool(v[2]) if v[2] >= 0 else None)} for v in vrows],
        }
        if args.sweep_unmask:
            # every geometry, interleaved round by round in this process; an
            # even number of passes per geometry leaves the batch masked, which
            # is verified byte-for-byte afterwards
            names, times = [], {}
            v = 0
            while L.hvws_set_unmask_variant(v) == 0:
                names.append((v, L.hvws_unmask_kernel_name().decode()))
                v += 1
            stimes = {}
            for _ in range(3):
                for v, name in names:
                    L.hvws_set_unmask_variant(v)
                    for _ in range(2):
                        eng.step(rx, plan.total, segs)
                        times.setdefault(name, []).append(eng.last_times()[1])
                    # the in-place STREAM ceiling with the same geometry (two passes: no net change)
                    eng.sync()
                    t = time.perf_counter()
                    for _ in range(2):
                        eng.stream_xor(rx, plan.total & ~15, 0x5A5A5A5A)
                    eng.sync()
                    stimes.setdefault(name, []).append((time.perf_counter() - t) / 2)
            L.hvws_set_unmask_variant(-1)
            ok = eng.synth(rx, plan.total, plan.seed, dp, 2 if passes % 2 else 1) == 0
            sweep = {n: (round(alg_bytes / (float(np.median(t)) * 1e-3) / 1e9, 1) if ok else None)
                     for n, t in times.items()}
            extra["unmask_sweep_GBps"] = sweep
            extra["stream_sweep_GBps"] = {n: round(2 * (plan.total & ~15) / float(np.median(t)) / 1e9, 1)
                                          for n, t in stimes.items()}
        extra["unmask_ms_mean"] = round(mean_unmask, 3)
        extra["unmask_events"] = ((f"HIP events on every {ev_every}th timed step" if ev_every > 1 else
                                   "HIP events on every timed step") +
                                  f" ({len(unmask_ms)} sampled of the last {len(times)})")

        # event loop, before the legs that allocate and
        # free large buffers: host-side rates measured after them ran slower
        if args.feed_conns > 0:
            extra["event_loop"], feed_streams, feed_pay = event_loop_leg(eng, device, args.feed_conns,
                                                                         args.feed_iters, plan.seed + 7)
        if args.dropin_reads > 0:
            extra["drop_in"] = dropin_leg_child(device, plan.seed + 11, args.dropin_reads)

    rx_plain = passes % 2 == 1   # payloads currently unmasked
    # host-inclusive: pinned host rx -> device -> scan+unmask -> host, every
    # rank at once (measured before the transmit leg: the pipeline's own
    # allocations ran measurably slower after that leg's 68.7 GB buffer came
    # and went)
    if dist is not None:
        dist.barrier()   # rank 0's extra legs above
    if args.host_gib > 0:
        res, sample = host_inclusive_leg(eng, plan, dp, rx, args, dist, rank, world, device)
        rx_plain = False
        if rank == 0:
            extra["host_inclusive"] = res

    if rank == 0 and not args.no_tx:
        extra["tx"] = tx_leg(eng, plan, dp, rx, rx_plain, segs, tpath)

    dp.free()
    rx.free()

    if rank == 0:
        cpu = None
        if sample is not None:
            ci = cpu_info()
            v1, kind, passes1, _ = cpu_baseline(sample, args.cpu_seconds, 1)
            nthr = ci["usable_cpus"]
            vn, _, _, _ = cpu_baseline(sample, args.cpu_seconds / 2, nthr)
            cpu = {
                "value": round(v1, 3), "unit": "GiB/s", "cores": 1, "kind": kind,
                "cpu_model": ci["cpu_model"], "nproc": ci["nproc"], "cgroup_cpus": ci["cgroup_cpus"],
                "sample": f"{sample.nbytes} B of the same batch ({args.config} frames) x {passes1} passes, "
                          "WebSocketParser semantics (header parse + in-place unmask + message append), 8 KiB chunks",
                "multi_thread": {"value": round(vn, 3), "threads": nthr,
                                 "note": "one independent stream per thread; threads = min(nproc, cgroup CPU quota)"},
                "decode_only": {"value": round(cpu_decode_only(sample, plan, args.cpu_seconds / 4), 3), "cores": 1,
                                "note": "websocket_decode over the sample's masked payload spans"},
                "note": "a reported baseline (the reference CPU path on this host), not the optimisation target",
            }
            if feed_streams is not None:
                cpu["event_loop"] = cpu_event_loop(feed_streams, args.feed_iters, feed_pay)
        out = {
            "metric": "device-resident WS unmask GiB/s, 64 KiB masked frames, 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (websocket_build_frame layout, splitmix64 payloads/keys, distinct seed per rank)",
            "config": {
                "workload": desc,
                "frames_per_gpu": plan.n,
                "rx_bytes_per_gpu": plan.total,
                "payload_bytes_per_gpu": plan.payload_bytes,
                "segments_per_gpu": segs.n,
                "parallelism": f"replicas{world} (disjoint batches, no collectives)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kname,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": alg_bytes,
                # boxes differ (in-place ceilings 5.4-6.6 TB/s across the pool): the
                # same kernel against this box's own STREAM-style ceiling, same buffer
                "frac_of_box_ceiling": (round(achieved / extra["stream_ceiling_GBps"], 4)
                                        if extra.get("stream_ceiling_GBps") else None),
            },
            "cpu_baseline": cpu,
        }
        out.update(extra)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
