"""GPU: batched FeedRecvData across connections --
an event loop's poll iteration hands every ready connection's read to one
GPU round trip; each connection must see exactly what the reference
WebSocketParser::FeedRecvData sequence produces."""
from __future__ import annotations

import ctypes
import os
import random

import pytest

import libhv_amd
import streams as S
import wsharness as H

pytestmark = pytest.mark.gpu

@pytest.fixture(params=["small", "small_copy", "general"], autouse=True)
def rx_path(request):
    """Run every case through the three host-batch paths: the single-launch
    small-batch kernel (default for reads this size; zero-copy for segments
    <= 32 KiB), the same kernel behind an H2D copy, and the general
    COUNT/EMIT/unmask sequence.  Results must be identical."""
    L = libhv_amd.lib()
    limit = 0 if request.param.startswith("small") else (1 << 64) - 1
    zc = 0 if request.param == "small_copy" else 1
    L.hvws_set_small_batch_limit(None, limit)
    L.hvws_set_small_zero_copy(None, zc)
    eng = request.getfixturevalue("eng") if "eng" in request.fixturenames else None
    if eng:
        L.hvws_set_small_batch_limit(eng.ctx, limit)
        L.hvws_set_small_zero_copy(eng.ctx, zc)
    yield request.param
    L.hvws_set_small_batch_limit(None, 0)
    L.hvws_set_small_zero_copy(None, 1)
    if eng:
        L.hvws_set_small_batch_limit(eng.ctx, 0)
        L.hvws_set_small_zero_copy(eng.ctx, 1)


def _clamp(chunks, n):
    """chunk sizes that exactly cover n bytes (rand_chunks may overshoot)"""
    out, at = [], 0
    for c in chunks:
        if at >= n:
            break
        c = min(c, n - at)
        out.append(c)
        at += c
    return out


class Conn:
    def __init__(self, data: bytes, chunks):
        self.data = data
        self.chunks = _clamp(chunks, len(data))
        self.fed = list(self.chunks)
        self.at = 0
        self.buf = ctypes.create_string_buffer(data, max(len(data), 1))
        L = libhv_amd.lib()
        self.h = L.hvws_wsp_new()
        self.sink = H.MsgLog()
        self.cb = libhv_amd.MSG_CB(self.sink._on)
        L.hvws_wsp_set_sink(self.h, self.cb, None)
        self.rets = []


def _loop(rng, conns, max_batch=None, dup=False, feeder=False):
    """One poll iteration per pass: the ready connections' next reads go to
    hvws_wsp_feed_many, or (feeder=True) to a pipelined hvws_feeder, whose
    rets for a submission arrive during the next submit or the final flush."""
    L = libhv_amd.lib()
    f = None
    if feeder:
        # "inline": every submission's device half on the loop thread (the
        # $HVWS_EXPERIMENT feeder_inline path, read when the feeder is made)
        if feeder == "inline":
            os.environ["HVWS_EXPERIMENT"] = f"feeder_inline={1 << 40}"
        f = L.hvws_feeder_new()
        os.environ.pop("HVWS_EXPERIMENT", None)
    subs = []
    pending = [c for c in conns if c.chunks]
    while pending:
        ready = [c for c in pending if rng.random() < 0.7] or pending[:1]
        if dup:   # a connection may be ready twice in one iteration
            ready = ready + [c for c in ready if rng.random() < 0.3 and len(c.chunks) > 1]
        if max_batch:
            ready = ready[:max_batch]
        n = len(ready)
        hs = (ctypes.c_void_p * n)()
        ds = (ctypes.c_void_p * n)()
        ls = (ctypes.c_size_t * n)()
        for i, c in enumerate(ready):
            k = c.chunks.pop(0)
            hs[i] = c.h
            ds[i] = ctypes.addressof(c.buf) + c.at
            ls[i] = k
            c.at += k
        rets = (ctypes.c_int * n)()
        if f:
            assert L.hvws_wsp_feeder_submit(f, hs, ds, ls, n, rets) == n
        else:
            assert L.hvws_wsp_feed_many(hs, ds, ls, n, rets) == n
        subs.append((ready, rets))
        pending = [c for c in conns if c.chunks]
    if f:
        assert L.hvws_feeder_flush(f) == 0
        L.hvws_feeder_free(f)
    for ready, rets in subs:
        for i, c in enumerate(ready):
            c.rets.append(rets[i])


def _check(conns):
    L = libhv_amd.lib()
    for c in conns:
        exp_msgs, exp_rets, exp_state, exp_buf = H.run_messages("oracle", c.data, c.fed)
        st = (ctypes.c_uint64 * 8)()
        L.hvws_wsp_state(c.h, st)
        assert c.sink.msgs == exp_msgs
        assert c.rets == exp_rets
        assert tuple(st) == exp_state
        assert c.buf.raw[:len(c.data)] == exp_buf
        L.hvws_wsp_free(c.h)


@pytest.mark.parametrize("feeder", [False, True, "inline"], ids=["many", "feeder", "feeder_inline"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_feed_many_matches_sequential_reference(seed, feeder):
    rng = random.Random(seed)
    conns = []
    for _ in range(rng.randint(5, 60)):
        data = S.rand_stream(rng, rng.randint(1, 15), max_len=rng.choice([60, 600, 70000]))
        chunks = S.rand_chunks(rng, len(data), rng.choice(["rand", "small", "one"]))
        c = Conn(data, chunks)
        conns.append(c)
    _loop(rng, conns, feeder=feeder)
    _check(conns)


@pytest.mark.parametrize("feeder", [False, True, "inline"], ids=["many", "feeder", "feeder_inline"])
def test_feed_many_repeated_connection_in_batch(feeder):
    rng = random.Random(9)
    conns = []
    for _ in range(12):
        data = S.rand_stream(rng, rng.randint(2, 10), max_len=300)
        chunks = S.rand_chunks(rng, len(data), "small")
        c = Conn(data, chunks)
        conns.append(c)
    _loop(rng, conns, dup=True, feeder=feeder)
    _check(conns)


def test_feed_many_config1_event_loop():
    """Config 1 (1000 x 1 KiB text) spread over 16 connections, 8 KiB reads."""
    from libhv_amd import synth

    plan = synth.config_plan("c1", seed=1).split(16)
    host = H.synth_cpu(plan)
    conns = []
    for off, n in plan.segments:
        data = host[off:off + n].tobytes()
        chunks = [8192] * (n // 8192) + ([n % 8192] if n % 8192 else [])
        c = Conn(data, chunks)
        conns.append(c)
    _loop(random.Random(4), conns)
    _check(conns)
    assert sum(len(c.sink.msgs) for c in conns) == 1000


def test_feed_many_reentrant_callback():
    """An onMessage that feeds another connection on the same loop thread
    (which restages, and here regrows, the thread's pinned stage) while the
    outer batch is still being replayed: every connection, the inner one
    included, must still see exactly the reference's results."""
    L = libhv_amd.lib()
    rng = random.Random(21)
    conns = []
    for _ in range(8):
        data = S.rand_stream(rng, rng.randint(4, 10), max_len=2000)
        conns.append(Conn(data, [len(data)]))
    inner_data = S.rand_stream(rng, 30, max_len=70000)   # larger than the outer batch
    inner = Conn(inner_data, [len(inner_data)])
    fired = []

    def on0(user, op, data, n):
        conns[0].sink._on(user, op, data, n)
        if not fired:
            fired.append(1)
            hs = (ctypes.c_void_p * 1)(inner.h)
            ds = (ctypes.c_void_p * 1)(ctypes.addressof(inner.buf))
            ls = (ctypes.c_size_t * 1)(len(inner.data))
            rets = (ctypes.c_int * 1)()
            assert L.hvws_wsp_feed_many(hs, ds, ls, 1, rets) == 1
            inner.rets.append(rets[0])
            inner.chunks = []

    conns[0].cb = libhv_amd.MSG_CB(on0)
    L.hvws_wsp_set_sink(conns[0].h, conns[0].cb, None)
    # every connection ready in the same poll iteration, connection 0 first
    n = len(conns)
    hs = (ctypes.c_void_p * n)(*[c.h for c in conns])
    ds = (ctypes.c_void_p * n)(*[ctypes.addressof(c.buf) for c in conns])
    ls = (ctypes.c_size_t * n)(*[len(c.data) for c in conns])
    rets = (ctypes.c_int * n)()
    assert L.hvws_wsp_feed_many(hs, ds, ls, n, rets) == n
    for i, c in enumerate(conns):
        c.rets.append(rets[i])
    assert fired, "connection 0 delivered no message"
    _check(conns + [inner])


@pytest.mark.parametrize("feeder", [False, True], ids=["many", "feeder"])
def test_feed_many_large_poll_iteration(feeder):
    """Poll iterations of ~2 MiB (256 connections x 8 KiB reads): the gather
    into and scatter out of the pinned stage split over the host copy pool
    (hvws_hostpool.cpp, batches >= 1 MiB).  Chunks land back in the right
    connections' buffers and every connection matches the reference."""
    rng = random.Random(31)
    conns = []
    for _ in range(256):
        data = S.rand_stream(rng, rng.randint(4, 12), max_len=rng.choice([600, 9000]))
        chunks = [8192] * (len(data) // 8192) + ([len(data) % 8192] if len(data) % 8192 else [])
        conns.append(Conn(data, chunks))
    _loop(random.Random(5), conns, feeder=feeder)
    assert sum(len(c.data) for c in conns) > 2 << 20
    _check(conns)


@pytest.mark.parametrize("read", [8192, 32768, 8191])
def test_feed_many_record_density(read):
    """k_small's XOR paths by records per segment: few long payloads (record-
    major), a few hundred (chunk-major, records in LDS) and more than its LDS
    record area holds (tiny frames, records in the device slot); reads of
    8191 bytes put segment ends and starts inside 16-byte chunks."""
    rng = random.Random(read)
    conns = []
    for max_len in (3000, 40, 4):
        for _ in range(4):
            data = S.rand_stream(rng, rng.randint(40, 3000) if max_len < 100 else rng.randint(10, 40),
                                 max_len=max_len)
            chunks = [read] * (len(data) // read) + ([len(data) % read] if len(data) % read else [])
            conns.append(Conn(data, chunks))
    _loop(random.Random(read + 1), conns)
    _check(conns)


@pytest.mark.parametrize("feeder", [False, True], ids=["many", "feeder"])
def test_nested_feed_of_parser_still_to_replay_refused(feeder):
    """An onMessage that feeds a parser whose state a replay still to come on
    this thread will write -- later in the same run, or in a feeder's run
    already in flight -- is refused (-1; libhv closes such a connection)
    instead of being overwritten silently.  Feeding any other parser works,
    and every connection still matches the reference."""
    L = libhv_amd.lib()
    rng = random.Random(61)
    a, b, c = (Conn(S.rand_stream(rng, 4, max_len=300), [0]) for _ in range(3))
    got = []

    def on_a(user, op, data, n):
        a.sink._on(user, op, data, n)
        if got:
            return
        def one(conn):
            hs = (ctypes.c_void_p * 1)(conn.h)
            ds = (ctypes.c_void_p * 1)(ctypes.addressof(conn.buf))
            ls = (ctypes.c_size_t * 1)(len(conn.data))
            rets = (ctypes.c_int * 1)()
            return L.hvws_wsp_feed_many(hs, ds, ls, 1, rets), rets[0]
        got.append(one(b))                                                   # still to replay: refused
        got.append(L.hvws_wsp_feed(b.h, ctypes.addressof(b.buf), len(b.data)))   # same through FeedRecvData
        got.append(one(c))                                                   # not in flight: fed

    a.cb = libhv_amd.MSG_CB(on_a)
    L.hvws_wsp_set_sink(a.h, a.cb, None)

    def sub(f, conns):
        n = len(conns)
        hs = (ctypes.c_void_p * n)(*[x.h for x in conns])
        ds = (ctypes.c_void_p * n)(*[ctypes.addressof(x.buf) for x in conns])
        ls = (ctypes.c_size_t * n)(*[len(x.data) for x in conns])
        rets = (ctypes.c_int * n)()
        if f:
            assert L.hvws_wsp_feeder_submit(f, hs, ds, ls, n, rets) == n
        else:
            assert L.hvws_wsp_feed_many(hs, ds, ls, n, rets) == n
        return rets

    if feeder:
        f = L.hvws_feeder_new()
        ra = sub(f, [a])
        rb = sub(f, [b])     # a's callbacks replay here, with b's run in flight
        assert L.hvws_feeder_flush(f) == 0
        L.hvws_feeder_free(f)
        rets = [ra[0], rb[0]]
    else:
        r = sub(None, [a, b])
        rets = [r[0], r[1]]
    assert got[0][0] == -1 and got[1] == -1 and got[2] == (1, len(c.data)), got
    for conn, r in zip((a, b, c), rets + [got[2][1]]):
        conn.fed, conn.rets = [len(conn.data)], [r]
    _check([a, b, c])


def test_feeder_free_from_callback():
    """hvws_feeder_free from inside one of the feeder's own callbacks is
    deferred until the flush that replays it returns: the rest of that run's
    callbacks still run, and nothing is used after the free."""
    L = libhv_amd.lib()
    rng = random.Random(71)
    conns = [Conn(S.rand_stream(rng, 5, max_len=400), [0]) for _ in range(6)]
    f = L.hvws_feeder_new()
    freed = []

    def on0(user, op, data, n):
        conns[0].sink._on(user, op, data, n)
        if not freed:
            freed.append(1)
            L.hvws_feeder_free(f)

    conns[0].cb = libhv_amd.MSG_CB(on0)
    L.hvws_wsp_set_sink(conns[0].h, conns[0].cb, None)
    n = len(conns)
    hs = (ctypes.c_void_p * n)(*[c.h for c in conns])
    ds = (ctypes.c_void_p * n)(*[ctypes.addressof(c.buf) for c in conns])
    ls = (ctypes.c_size_t * n)(*[len(c.data) for c in conns])
    rets = (ctypes.c_int * n)()
    assert L.hvws_wsp_feeder_submit(f, hs, ds, ls, n, rets) == n
    assert L.hvws_feeder_flush(f) == 0   # replays; the callback frees f, which happens on return
    assert freed
    for i, c in enumerate(conns):
        c.fed, c.rets = [len(c.data)], [rets[i]]
    _check(conns)


def test_feeder_callbacks_one_submission_late():
    """A feeder replays submission k's callbacks during submit k+1 (or flush):
    nothing is delivered by the first submit, everything by the flush; a
    submit from inside one of its own callbacks is refused (-1)."""
    L = libhv_amd.lib()
    rng = random.Random(41)
    conns = [Conn(S.rand_stream(rng, 6, max_len=500), [0]) for _ in range(5)]
    f = L.hvws_feeder_new()
    inner = []

    def on0(user, op, data, n):
        conns[0].sink._on(user, op, data, n)
        if not inner:
            h = (ctypes.c_void_p * 1)(conns[1].h)
            d = (ctypes.c_void_p * 1)(ctypes.addressof(conns[1].buf))
            ln = (ctypes.c_size_t * 1)(1)
            inner.append(L.hvws_wsp_feeder_submit(f, h, d, ln, 1, None))
            inner.append(L.hvws_feeder_flush(f))

    conns[0].cb = libhv_amd.MSG_CB(on0)
    L.hvws_wsp_set_sink(conns[0].h, conns[0].cb, None)
    n = len(conns)
    hs = (ctypes.c_void_p * n)(*[c.h for c in conns])
    ds = (ctypes.c_void_p * n)(*[ctypes.addressof(c.buf) for c in conns])
    ls = (ctypes.c_size_t * n)(*[len(c.data) for c in conns])
    rets = (ctypes.c_int * n)()
    assert L.hvws_wsp_feeder_submit(f, hs, ds, ls, n, rets) == n
    assert all(not c.sink.msgs for c in conns) and list(rets) == [0] * n
    assert L.hvws_wsp_feeder_submit(f, hs, ds, ls, 0, None) == 0   # 0 reads = flush
    assert inner == [-1, -1]
    for i, c in enumerate(conns):
        c.fed = [len(c.data)]
        c.rets = [rets[i]]
    L.hvws_feeder_free(f)
    _check(conns)
