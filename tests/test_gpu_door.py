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
import os
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


@pytest.mark.skipif(os.environ.get("HVWS_DOOR", "1") == "0", reason="$HVWS_DOOR=0 turns the default off")
def test_door_is_the_default():
    """Round 4: a thread's first reference-API read goes to the resident
    worker without hvws_set_door (a launch per call only when asked for)."""
    def first_read():
        L = libhv_amd.lib()
        assert L.hvws_set_door(None, -1) == 1   # nothing set on this thread's context: the default, on
        before = _stats()
        data = S.rand_stream(random.Random(5), 6, max_len=3000)
        assert H.run_messages("gpu", data, [len(data)]) == H.run_messages("oracle", data, [len(data)])
        after = _stats()
        assert after[1] > before[1], "the read did not go to the worker"
        L.hvws_thread_release()

    _in_thread(first_read)
    assert _health() == (0, 0), "a worker stream wedged or a request went unanswered (stderr has the mailbox)"


def _health():
    out = (ctypes.c_uint64 * 2)()
    assert libhv_amd.lib().hvws_door_health(out) == 0
    return int(out[0]), int(out[1])


def test_door_many_threads_capped():
    """24 loop threads at once (advisor r4): at most $HVWS_DOOR_MAX (8) of
    them hold a worker stream on the device -- each is a hardware queue of its
    own -- and the rest launch per call; every thread's messages equal the
    oracle's, and no worker wedges or leaves a request unanswered."""
    n = 24
    work = [_cases(random.Random(100 + i), 6) for i in range(n)]
    fed = threading.Barrier(n + 1, timeout=120)
    done = threading.Event()
    has_stream, errs = [0] * n, []

    def loop(i):
        L = libhv_amd.lib()
        try:
            for data, chunks in work[i]:
                if H.run_messages("gpu", data, chunks) != H.run_messages("oracle", data, chunks):
                    errs.append(f"thread {i}: mismatch")
            info = (ctypes.c_uint64 * 2)()
            L.hvws_door_info(None, info)
            has_stream[i] = int(info[1])
        except Exception as e:   # noqa: BLE001
            errs.append(f"thread {i}: {e!r}")
        finally:
            try:
                fed.wait()          # every thread has fed: count the streams held at once
                done.wait(120)
            finally:
                L.hvws_thread_release()

    ths = [threading.Thread(target=loop, args=(i,)) for i in range(n)]
    for t in ths:
        t.start()
    fed.wait()
    held = sum(has_stream)
    done.set()
    for t in ths:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ths), "a loop thread did not finish"
    assert not errs, errs
    assert 1 <= held <= 8, f"{held} loop threads hold a worker stream at once (cap 8)"
    assert _health() == (0, 0)


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


def test_door_carried_payload_every_alignment(door):
    """Reads of 8 KiB + k bytes (k = 0..15) over masked frames of 1000-1100 B:
    almost every read starts inside a payload, which the worker unmasks while
    its header walk reads the next frame's header, and that payload's end --
    the chunk its last bytes share with the header -- falls at every alignment.
    Messages, return values and the in-place buffer equal the oracle's."""
    rng = random.Random(23)
    frames = [(0x2 | S.FIN | S.MASK, rng.randbytes(rng.randint(1000, 1100)), rng.randbytes(4)) for _ in range(200)]
    data = H.build_frames_ref(frames)
    chunks, tot, k = [], 0, 0
    while tot < len(data):
        chunks.append(min(8192 + k % 16, len(data) - tot))
        tot += chunks[-1]
        k += 1
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


def _in_thread(fn, timeout=120):
    """fn() on a new thread (its own reference-API context); re-raises its
    exception here."""
    err = []

    def run():
        try:
            fn()
        except BaseException as e:   # noqa: BLE001
            err.append(e)

    t = threading.Thread(target=run)
    t.start()
    t.join(timeout=min(timeout, 60))
    if t.is_alive():
        # leave the native stacks and every context's mailbox on stderr
        L = libhv_amd.lib()
        L.hvws_debug_backtraces(2)
        L.hvws_debug_dump(2)
    assert not t.is_alive(), "thread did not finish"
    if err:
        raise err[0]


def test_door_free_on_another_thread_parks_the_worker():
    """A free on one thread while another thread's worker is resident: the
    runtime's hipFree waits for every stream of the device, the worker's
    too, so the library parks every worker of the device before its own
    frees (round 3 parked only the calling thread's; with a 10 s idle time
    this free would then have waited ~10 s).  The owner's next call
    relaunches its worker; results stay the oracle's."""
    L = libhv_amd.lib()
    resident = threading.Event()
    freed = threading.Event()
    out = {}
    rng = random.Random(41)
    cases = _cases(rng, 6)

    def owner():
        old_idle = L.hvws_set_door_idle_us(10_000_000)
        L.hvws_set_door(None, 1)
        try:
            data, chunks = cases[0]
            assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks)
            out["before"] = _stats()
            resident.set()
            assert freed.wait(60)
            out["after_free"] = _stats()
            for data, chunks in cases[1:]:
                assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks)
            out["end"] = _stats()
        finally:
            L.hvws_set_door(None, 0)
            L.hvws_set_door_idle_us(old_idle)
            L.hvws_thread_release()

    errs = []

    def run_owner():
        try:
            owner()
        except BaseException as e:   # noqa: BLE001
            errs.append(e)

    t = threading.Thread(target=run_owner)
    t.start()
    try:
        assert resident.wait(60), errs
        assert out["before"][3] == 1, "the worker is not resident"
        with libhv_amd.Engine(0) as eng:
            t0 = time.perf_counter()
            p = L.hvws_dev_alloc(eng.ctx, 1 << 20)
            L.hvws_dev_free(eng.ctx, p)
            h = L.hvws_host_alloc(eng.ctx, 1 << 20)
            L.hvws_host_free(eng.ctx, h)
            dt = time.perf_counter() - t0
    finally:
        freed.set()
        t.join(120)
    assert not errs, errs
    assert dt < 2.0, f"frees beside another thread's resident worker took {dt:.2f} s"
    assert out["after_free"][3] == 0, "the free did not park the other thread's worker"
    assert out["end"][0] > out["before"][0], "the owner's next call did not relaunch its worker"


def test_door_bench_sequence():
    """bench.py's sequence when its drop-in leg ran (two of four such runs
    hung in round 3, profiles/r3ae_raw): a thread context with the worker on
    serves FeedRecvData and masked websocket_build_frame calls, switches it
    off and on between passes, goes back to the default (-1) and releases
    its context; then a feeder with registered pinned reads and a batched
    feed; then hvws_pipeline calls (with their allocations and frees) on an
    explicit context -- each call bounded, every result checked."""
    from libhv_amd import synth

    L = libhv_amd.lib()
    rng = random.Random(71)
    cases = _cases(rng, 8)

    def dropin():
        key = b"\x12\x34\x56\x78"
        payload = bytes(range(125))
        for rnd in range(3):
            for on in (1, 0):
                L.hvws_set_door(None, on)
                for data, chunks in cases:
                    assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks)
                for _ in range(50):
                    buf = ctypes.create_string_buffer(256)
                    n = L.websocket_build_frame(buf, 0x2 | 0x10 | 0x20, key, payload, 125)
                    assert buf.raw[:n] == H.build_frames_ref([(0x32, payload, key)])
        L.hvws_set_door(None, 0)   # off parks the worker now
        st = _stats()
        assert st[3] == 0, "the worker is still resident after hvws_set_door(0)"
        L.hvws_set_door(None, -1)   # back to the default (on) without a relaunch
        L.hvws_thread_release()

    t0 = time.perf_counter()
    _in_thread(dropin)
    t_dropin = time.perf_counter() - t0

    # event loop: a feeder over registered pinned reads, then a batched feed
    conns, per = 16, 8192
    fp = synth.uniform_plan(conns * (per * 3 // 1032 + 2), 1024, 5).split(conns)
    host = H.synth_cpu(fp)
    streams = [host[o:o + 3 * per] for o, _ in fp.segments]
    with libhv_amd.Engine(0) as eng:
        arena = L.hvws_host_alloc(eng.ctx, conns * 3 * per)
        try:
            ring = np.ctypeslib.as_array((ctypes.c_uint8 * (conns * 3 * per)).from_address(arena))
            for i, s in enumerate(streams):
                ring[i * 3 * per:(i + 1) * 3 * per] = s
            f = L.hvws_feeder_new()
            hs = [L.hvws_wsp_new() for _ in range(conns)]
            hv = (ctypes.c_void_p * conns)(*hs)
            lens = (ctypes.c_size_t * conns)(*([per] * conns))
            rets = (ctypes.c_int * conns)()
            for it in range(3):
                ds = (ctypes.c_void_p * conns)(*[arena + i * 3 * per + it * per for i in range(conns)])
                if it < 2:
                    assert L.hvws_wsp_feeder_submit(f, hv, ds, lens, conns, rets) == conns
                else:
                    assert L.hvws_feeder_flush(f) == 0
                    assert L.hvws_wsp_feed_many(hv, ds, lens, conns, rets) == conns
                    assert list(rets) == [per] * conns
            L.hvws_feeder_free(f)
            for h in hs:
                L.hvws_wsp_free(h)
        finally:
            L.hvws_host_free(eng.ctx, arena)

        # host-inclusive pipeline on the explicit context, toggling the bytes
        plan = synth.mixed_plan(24 << 20, 33, hi=1 << 19)
        hb = H.synth_cpu(plan)
        _, _, _, exp = _oracle_batch_one(hb)
        pinned = L.hvws_host_alloc(eng.ctx, plan.total)
        try:
            arr = np.ctypeslib.as_array((ctypes.c_uint8 * plan.total).from_address(pinned))
            arr[:] = hb
            for r in range(4):
                carry = libhv_amd.WsParser()
                L.websocket_parser_init(ctypes.byref(carry))
                t = time.perf_counter()
                assert L.hvws_pipeline(eng.ctx, pinned, plan.total, 4 << 20, ctypes.byref(carry)) == 0, \
                    L.hvws_last_error()
                assert time.perf_counter() - t < 10, f"pipeline call {r} took {time.perf_counter() - t:.1f} s"
                assert np.array_equal(arr, exp if r % 2 == 0 else hb), r
        finally:
            L.hvws_host_free(eng.ctx, pinned)
    assert t_dropin < 60


def _oracle_batch_one(buf):
    """The oracle's frames and unmasked bytes of one stream."""
    import test_gpu_parity as P

    return P._oracle_batch(buf, [(0, len(buf))], None)


@pytest.mark.parametrize("release", [False, True])
def test_child_process_with_worker_exits_cleanly(release):
    """a process whose reference-API read went to the
    resident worker exits with status 0 -- its worker asked home and its
    worker queue destroyed by the exit handler (hvws_doorq.cpp), whether the
    thread's context was released first or not (scripts/probe/exit_probe.py,
    run as a child process as a libhv server process would run)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, EXIT_PROBE_MAPS="0", EXIT_PROBE_RELEASE="1" if release else "0")
    env.pop("HVWS_DOOR", None)
    p = subprocess.run([sys.executable, os.path.join(root, "scripts", "probe", "exit_probe.py"), "test"], env=env,
                       capture_output=True, text=True, timeout=90)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    assert "the read went to the worker" in p.stdout


def test_door_request_in_pinned_host_memory():
    """The worker's request block and bytes in pinned host memory ($HVWS_EXPERIMENT
    door_vram=0: the layout of a box without a large BAR), polled across PCIe
    with the block's seq_tail check: feeds, decodes and masked builds in a
    child process equal the oracle's (tests/door_pinned_child.py)."""
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, HVWS_EXPERIMENT="door_vram=0")
    env.pop("HVWS_DOOR", None)
    p = subprocess.run([sys.executable, os.path.join(here, "door_pinned_child.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    assert p.stdout.startswith("ok "), p.stdout
