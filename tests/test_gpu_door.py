"""GPU: the resident small-path worker (k_door, hvws_set_door).  The
reference API's single calls -- WebSocketParser::FeedRecvData and
websocket_parser_execute on one read (http/WebSocketParser.cpp:73-75,
http/websocket_parser.c:53-171), websocket_decode / websocket_parser_decode
(:173-189) and a masked websocket_build_frame (:207-256) -- are served by one
workgroup that stays on the device between calls.  Every result must equal
the oracle's (and the per-launch path's) byte for byte, through parking and
relaunching, and the resident kernel must hold up no other work."""
from __future__ import annotations

import ctypes
import random
import threading
import time

import numpy as np
import pytest

import libhv_amd
import streams as S
import wsharness as H

pytestmark = pytest.mark.gpu


def _stats():
    out = (ctypes.c_uint64 * 4)()
    assert libhv_amd.lib().hvws_door_stats(None, out) == 0
    return list(out)


@pytest.fixture
def door():
    L = libhv_amd.lib()
    old = L.hvws_set_door(None, 1)
    yield L
    L.hvws_set_door(None, old)
    L.hvws_set_door_idle_us(0)


def _cases(rng, n):
    out = []
    for _ in range(n):
        data = S.rand_stream(rng, rng.randint(1, 14), max_len=rng.choice([30, 300, 3000, 9000]))
        out.append((data, S.rand_chunks(rng, len(data), rng.choice(["rand", "small", "one"]))))
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_door_messages_match_oracle(door, seed):
    """FeedRecvData read by read (reads <= 32 KiB go to the worker): messages,
    return values, final state and the in-place buffer equal the oracle's;
    the same again with the worker off."""
    rng = random.Random(seed)
    before = _stats()
    for data, chunks in _cases(rng, 40):
        exp = H.run_messages("oracle", data, chunks)
        assert H.run_messages("gpu", data, chunks) == exp
    assert _stats()[1] > before[1], "no request reached the worker"
    door.hvws_set_door(None, 0)   # parks the worker (one last request: its exit)
    st = _stats()
    for data, chunks in _cases(random.Random(seed), 10):
        assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks)
    assert _stats()[1] == st[1]   # worker off: no request posted


def test_door_varying_read_sizes(door):
    """Consecutive reads through one worker that grow, shrink and repeat
    (1 B .. 32 KiB, the worker's largest request) all equal the oracle's."""
    rng = random.Random(17)
    data = S.rand_stream(rng, 120, max_len=3000)
    sizes = [100, 32768, 5, 20000, 8192, 1, 32768, 32767, 16, 8192, 8192, 9000, 3]
    chunks, tot = [], 0
    for c in sizes * 4:
        if tot >= len(data):
            break
        chunks.append(min(c, len(data) - tot))
        tot += chunks[-1]
    if tot < len(data):
        chunks.append(len(data) - tot)
    before = _stats()
    assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks)
    assert _stats()[1] > before[1], "no request reached the worker"


def test_door_execute_callbacks_and_early_return(door):
    """websocket_parser_execute through the worker: callback logs (with and
    without the user's in-callback decode) and early returns equal the oracle's."""
    rng = random.Random(5)
    for t in range(60):
        data = S.rand_stream(rng, rng.randint(1, 10), max_len=rng.choice([20, 300, 5000]))
        chunks = S.rand_chunks(rng, len(data), rng.choice(["rand", "small", "one"]))
        abort_at = rng.choice([-1, -1, rng.randint(0, 10)])
        dec = rng.random() < 0.5
        assert H.run_evlog("gpu", data, chunks, abort_at, dec) == H.run_evlog("oracle", data, chunks, abort_at, dec)


def test_door_decode_and_build_frame(door):
    """websocket_decode at every phase and length around the chunk size, and
    masked websocket_build_frame (the XOR request) against the oracle."""
    L, O = door, H.oracle()
    rng = random.Random(9)
    for n in list(range(0, 40)) + [125, 126, 4095, 4096, 4097, 32767, 32768, 32769, 70000]:
        src = rng.randbytes(n)
        key = rng.randbytes(4)
        for phase in range(4):
            a = ctypes.create_string_buffer(n + 1)
            b = ctypes.create_string_buffer(n + 1)
            ra = L.websocket_decode(a, src, n, key, phase)
            rb = O.ows_decode(b, src, n, key, phase)
            assert ra == rb and a.raw[:n] == b.raw[:n], (n, phase)
        for fl in (0x1 | 0x10 | 0x20, 0x2 | 0x20):
            out = ctypes.create_string_buffer(n + 16)
            m = L.websocket_build_frame(out, fl, key, src, n)
            assert out.raw[:m] == H.build_frames_ref([(fl, src, key)])


def test_door_parks_and_relaunches(door):
    """A worker idle for longer than its idle time parks; the next call
    relaunches it.  Calls spaced around the idle time (a request may arrive
    while the worker is parking) all return the oracle's results."""
    L = door
    L.hvws_set_door(None, 0)   # park the current worker: the new idle time applies to the next launch
    L.hvws_set_door(None, 1)
    L.hvws_set_door_idle_us(300)
    rng = random.Random(13)
    cases = _cases(rng, 120)
    l0 = _stats()[0]
    for i, (data, chunks) in enumerate(cases):
        time.sleep(rng.choice([0, 0, 0.0001, 0.0002, 0.0003, 0.0004, 0.002]))
        assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks), i
    assert _stats()[0] > l0 + 2, "the worker never parked and relaunched"


def test_door_holds_up_no_other_work(door):
    """While the worker is resident (idle time 1 s here), work on the other
    streams -- the same thread's context for a read too large for the worker
    (k_small on the context stream), and another context's step -- runs at
    once: the worker has a hardware queue of its own.  (Buffers are grown
    before the worker starts: the runtime's frees wait for every stream, the
    worker's too, so growing one parks the calling thread's worker first.)"""
    L = door
    from libhv_amd import synth

    big = S.rand_stream(random.Random(4), 30, max_len=20000)   # > 32 KiB: not the worker's
    assert len(big) > 32 << 10
    exp_big = H.run_messages("oracle", big, [len(big)])
    plan = synth.uniform_plan(2000, 1024, 3).split(8)
    host = H.synth_cpu(plan)
    with libhv_amd.Engine(0) as eng:
        rx = eng.to_device(host)
        L.hvws_set_door(None, 0)
        for _ in range(2):   # grow this thread's buffers and the other context's (both table sets)
            assert H.run_messages("gpu", big, [len(big)]) == exp_big
            eng.step(rx, plan.total, plan.segments)
        eng.sync()
        L.hvws_set_door(None, 1)
        L.hvws_set_door_idle_us(1_000_000)
        try:
            data = S.rand_stream(random.Random(3), 3, max_len=500)
            assert H.run_messages("gpu", data, [len(data)]) == H.run_messages("oracle", data, [len(data)])
            assert _stats()[3] == 1   # resident
            t = time.perf_counter()
            got = H.run_messages("gpu", big, [len(big)])
            dt1 = time.perf_counter() - t
            t = time.perf_counter()
            eng.step(rx, plan.total, plan.segments)
            eng.sync()
            dt2 = time.perf_counter() - t
            assert got == exp_big
            assert dt1 < 0.2, f"a read on the same context beside the resident worker took {dt1:.3f} s"
            assert dt2 < 0.2, f"a step on another context beside the resident worker took {dt2:.3f} s"
            assert _stats()[3] == 1, "the worker was parked (a buffer grew)"
        finally:
            L.hvws_set_door(None, 0)   # park (idle time 1 s)
            L.hvws_set_door_idle_us(0)
            rx.free()


def test_door_per_thread_workers():
    """Several loop threads, each with its own context and worker, feed at
    once; a thread that exits parks its worker (no hang at the end)."""
    rng = random.Random(17)
    work = [_cases(random.Random(rng.random()), 25) for _ in range(4)]
    errs = []

    def loop(cases):
        try:
            libhv_amd.lib().hvws_set_door(None, 1)   # this thread's context (the worker is opt-in)
            for data, chunks in cases:
                if H.run_messages("gpu", data, chunks) != H.run_messages("oracle", data, chunks):
                    errs.append("mismatch")
            out = (ctypes.c_uint64 * 4)()
            libhv_amd.lib().hvws_door_stats(None, out)
            if out[1] == 0:
                errs.append("thread posted no request")
        except Exception as e:   # noqa: BLE001
            errs.append(repr(e))

    ths = [threading.Thread(target=loop, args=(w,)) for w in work]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errs, errs


def test_door_validation_rejects_like_per_launch_path(door):
    """hvws_set_validation on the thread context applies to the worker: the
    same return values and states as with the worker off."""
    L = door
    rng = random.Random(23)
    streams = []
    for _ in range(30):
        frames = []
        for _ in range(rng.randint(1, 6)):
            # reserved opcodes, a fragmented control frame, an unmasked frame
            fl = rng.choice([0x31, 0x32, 0x33, 0x3B, 0x29, 0x12, 0x32])
            frames.append((fl, rng.randbytes(rng.randint(0, 200)), rng.randbytes(4) if fl & 0x20 else None))
        streams.append(H.build_frames_ref(frames))
    old = L.hvws_set_validation(None, 0x3F)
    try:
        res = {}
        for on in (1, 0):
            L.hvws_set_door(None, on)
            res[on] = [H.run_messages("gpu", d, S.rand_chunks(random.Random(i), len(d), "small"))
                       for i, d in enumerate(streams)]
        assert res[1] == res[0]
    finally:
        L.hvws_set_validation(None, old)
