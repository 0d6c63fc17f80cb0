"""GPU: hvws_rx_reads -- an event loop's reads taken where they lie, in
registered pinned memory (hvws_host_alloc / hvws_host_register), with no
gather into a staging buffer and no write-back copy.  Every read must give
exactly the oracle's frame records (offsets relative to the read), carry-out
and unmasked bytes (http/websocket_parser.c:53-180 through
http/WebSocketParser.cpp:28-37), whatever order the reads come in; the
batched drop-in (hvws_feed_many, hvws_feeder) takes this path for such
buffers and must still match the reference connection by connection."""
from __future__ import annotations

import ctypes
import random

import numpy as np
import pytest

import libhv_amd
import streams as S
import wsharness as H
from test_gpu_feed_many import Conn, _check, _loop

pytestmark = pytest.mark.gpu

EINVAL = -2   # HVWS_EINVAL


def _arena(eng, nbytes):
    L = libhv_amd.lib()
    p = L.hvws_host_alloc(eng.ctx, nbytes)
    assert p, L.hvws_last_error()
    return p


def _cases(rng, n, max_read=8192):
    """n (prefix, read) pairs: the prefix of a random stream goes through the
    oracle to make the carry-in, the read is the next chunk (<= max_read)."""
    out = []
    for _ in range(n):
        data = S.rand_stream(rng, rng.randint(1, 12), max_len=rng.choice([40, 600, 3000]))
        cut = rng.randint(0, len(data))
        ln = min(rng.randint(0, max_read), len(data) - cut)
        out.append((data[:cut], data[cut:cut + ln]))
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("order", ["address", "shuffled"])
def test_rx_reads_match_oracle(eng, seed, order):
    L = libhv_amd.lib()
    rng = random.Random(seed * 7 + (order == "shuffled"))
    cases = _cases(rng, rng.randint(1, 300))
    # reads laid out in the arena with gaps and every alignment
    offs, at = [], 0
    for _, rd in cases:
        at += rng.randint(0, 40)
        offs.append(at)
        at += len(rd)
    base = _arena(eng, at + 64)
    try:
        idx = list(range(len(cases)))
        if order == "shuffled":
            rng.shuffle(idx)
        carries, exp = [], []
        for i in idx:
            pre, rd = cases[i]
            _, st, _, _ = H.scan_segment(pre)
            ctypes.memmove(base + offs[i], rd, len(rd))
            recs, st_out, started, buf = H.scan_segment(rd, st)
            carries.append(st)
            exp.append((recs, st_out, started, buf))
        n = len(idx)
        reads = (ctypes.c_void_p * n)(*[base + offs[i] for i in idx])
        lens = (ctypes.c_uint64 * n)(*[len(cases[i][1]) for i in idx])
        carry = (libhv_amd.WsParser * n)()
        for k, st in enumerate(carries):
            ctypes.memmove(ctypes.byref(carry[k]), ctypes.byref(st), ctypes.sizeof(st))
        assert L.hvws_rx_reads(eng.ctx, reads, lens, carry, n, 1) == 0, L.hvws_last_error()
        frames = eng.frames()
        first, count = eng.segment_frames(n)
        _, started = eng.carry(n)
        for k, i in enumerate(idx):
            recs, st_out, st_started, buf = exp[k]
            got = frames[int(first[k]):int(first[k] + count[k])]
            assert got.tobytes() == recs.tobytes(), f"read {k}"
            assert carry[k].fields() == st_out.fields(), f"read {k}"
            assert started[k] == st_started
            assert ctypes.string_at(base + offs[i], len(cases[i][1])) == buf, f"read {k}"
    finally:
        L.hvws_host_free(eng.ctx, base)


def test_rx_reads_registered_caller_memory(eng):
    """hvws_host_register pins memory the caller already has (numpy here);
    reads in it are unmasked in place; after unregister they are refused."""
    L = libhv_amd.lib()
    rng = random.Random(11)
    cases = _cases(rng, 40, max_read=4000)
    size = sum(len(r) for _, r in cases) + 4096
    arr = np.zeros(size, np.uint8)
    assert L.hvws_host_register(eng.ctx, arr.ctypes.data, arr.nbytes) == 0, L.hvws_last_error()
    try:
        at, ptrs, exp = 0, [], []
        carry = (libhv_amd.WsParser * len(cases))()
        for k, (pre, rd) in enumerate(cases):
            _, st, _, _ = H.scan_segment(pre)
            ctypes.memmove(ctypes.byref(carry[k]), ctypes.byref(st), ctypes.sizeof(st))
            arr[at:at + len(rd)] = np.frombuffer(rd, np.uint8)
            ptrs.append(at)
            exp.append(H.scan_segment(rd, st)[3])
            at += len(rd)
        n = len(cases)
        reads = (ctypes.c_void_p * n)(*[arr.ctypes.data + p for p in ptrs])
        lens = (ctypes.c_uint64 * n)(*[len(r) for _, r in cases])
        assert L.hvws_rx_reads(eng.ctx, reads, lens, carry, n, 1) == 0, L.hvws_last_error()
        for k in range(n):
            assert arr[ptrs[k]:ptrs[k] + len(cases[k][1])].tobytes() == exp[k]
    finally:
        assert L.hvws_host_unregister(eng.ctx, arr.ctypes.data) == 0
    reads = (ctypes.c_void_p * 1)(arr.ctypes.data)
    lens = (ctypes.c_uint64 * 1)(16)
    assert L.hvws_rx_reads(eng.ctx, reads, lens, None, 1, 1) == EINVAL


def test_rx_reads_rejects_bad_tables(eng):
    """Unregistered, overlapping and over-long reads are refused (nothing is
    touched); the batched drop-in then falls back to its staging path."""
    L = libhv_amd.lib()
    base = _arena(eng, 1 << 17)
    try:
        data = bytes(range(256)) * 64
        ctypes.memmove(base, data, len(data))
        page = np.zeros(4096, np.uint8)

        def call(ptrs, lens):
            r = (ctypes.c_void_p * len(ptrs))(*ptrs)
            ln = (ctypes.c_uint64 * len(lens))(*lens)
            return L.hvws_rx_reads(eng.ctx, r, ln, None, len(ptrs), 1)

        assert call([page.ctypes.data], [100]) == EINVAL                  # not registered
        assert call([base, base + 50], [100, 100]) == EINVAL              # overlap
        assert call([base + 200, base], [100, 201]) == EINVAL             # overlap, out of order
        assert call([base], [(32 << 10) + 1]) == EINVAL                   # longer than 32 KiB
        assert call([base + (1 << 17) - 8], [16]) == EINVAL               # runs past the range
        assert ctypes.string_at(base, len(data)) == data
        assert call([base, base + 100], [100, 100]) == 0, L.hvws_last_error()
    finally:
        L.hvws_host_free(eng.ctx, base)


class PinnedConn(Conn):
    """A connection whose stream sits in a slice of a pinned arena (the read
    buffers an event loop would allocate with hvws_host_alloc)."""

    def __init__(self, data, chunks, addr):
        super().__init__(data, chunks)
        self.buf = (ctypes.c_char * max(len(data), 1)).from_address(addr)
        ctypes.memmove(addr, data, len(data))


def test_rx_reads_refused_with_small_path_off(eng):
    """hvws_set_small_batch_limit(ctx, ~0) turns the small path off; reads in
    place exist only there, so hvws_rx_reads refuses and the batched drop-in
    falls back to the general path (test_feed_from_pinned_buffers[general])."""
    L = libhv_amd.lib()
    base = _arena(eng, 4096)
    try:
        r = (ctypes.c_void_p * 1)(base)
        ln = (ctypes.c_uint64 * 1)(100)
        old = L.hvws_set_small_batch_limit(eng.ctx, (1 << 64) - 1)
        assert L.hvws_rx_reads(eng.ctx, r, ln, None, 1, 1) == EINVAL
        L.hvws_set_small_batch_limit(eng.ctx, old)
        assert L.hvws_rx_reads(eng.ctx, r, ln, None, 1, 1) == 0, L.hvws_last_error()
    finally:
        L.hvws_host_free(eng.ctx, base)


@pytest.mark.parametrize("path", ["small", "general"])
@pytest.mark.parametrize("feeder", [False, True], ids=["many", "feeder"])
@pytest.mark.parametrize("seed", [1, 2])
def test_feed_from_pinned_buffers(eng, seed, feeder, path):
    L = libhv_amd.lib()
    L.hvws_set_small_batch_limit(None, 0 if path == "small" else (1 << 64) - 1)
    try:
        _feed_from_pinned(eng, seed, feeder)
    finally:
        L.hvws_set_small_batch_limit(None, 0)


def _feed_from_pinned(eng, seed, feeder):
    rng = random.Random(100 + seed)
    streams = []
    for _ in range(rng.randint(20, 120)):
        data = S.rand_stream(rng, rng.randint(1, 15), max_len=rng.choice([60, 600, 3000]))
        streams.append((data, S.rand_chunks(rng, len(data), rng.choice(["rand", "small"]))))
    size = sum(len(d) + 16 for d, _ in streams)
    base = _arena(eng, size)
    try:
        conns, at = [], 0
        for data, chunks in streams:
            conns.append(PinnedConn(data, chunks, base + at))
            at += len(data) + rng.randint(0, 16)
        _loop(rng, conns, feeder=feeder)
        _check(conns)
    finally:
        libhv_amd.lib().hvws_host_free(eng.ctx, base)
