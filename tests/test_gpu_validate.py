"""GPU, optional protocol validation (SURVEY.md sec. 8(f) row 4,
hvws_set_validation).  Off by default -- every other parity test runs with it
off and matches the reference.  On, the frame records carry the RFC 6455
violation classes computed by the spec oracle tests/wsvalidate.py, whatever
the batch/segment cuts (headers split across batches keep their partial
state in the parser's padding byte), and the reference API rejects the first
violating header the way a failing on_frame_header callback would."""
from __future__ import annotations

import ctypes
import random

import numpy as np
import pytest

import libhv_amd
import wsharness as H
import wsvalidate as V

pytestmark = pytest.mark.gpu
I_HDR, I_INVALID = 1 << 10, 1 << 14


@pytest.fixture(params=["small", "general"])
def path(request, eng):
    L = libhv_amd.lib()
    limit = 0 if request.param == "small" else (1 << 64) - 1
    L.hvws_set_small_batch_limit(eng.ctx, limit)
    L.hvws_set_small_batch_limit(None, limit)
    yield request.param
    L.hvws_set_small_batch_limit(eng.ctx, 0)
    L.hvws_set_small_batch_limit(None, 0)
    L.hvws_set_validation(eng.ctx, 0)
    L.hvws_set_validation(None, 0)


def _hdr_classes(frames):
    return [(int(f["info"]) >> 16) & 63 for f in frames if int(f["info"]) & I_HDR]


def _invalid_flags(frames):
    return [bool(int(f["info"]) & I_INVALID) for f in frames if int(f["info"]) & I_HDR]


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_classes_one_batch(eng, path, seed):
    data, exp = V.random_stream(seed, 300, tail_len64=True)
    assert [v for _, v in V.violations(data)] == exp
    L = libhv_amd.lib()
    for vmask in (V.V_ALL, V.V_RSV | V.V_UNMASKED, V.V_CONTROL | V.V_NONMIN | V.V_LEN64, 0):
        L.hvws_set_validation(eng.ctx, vmask)
        host = np.frombuffer(data, dtype=np.uint8).copy()
        eng.rx_batch(host, [(0, len(data))], None, True)
        fr = eng.frames()
        assert _hdr_classes(fr) == [v & vmask for v in exp]
        assert _invalid_flags(fr) == [bool(v & vmask) for v in exp]


def test_validation_off_is_reference(eng, path):
    data, _ = V.random_stream(9, 200)
    host_a = np.frombuffer(data, dtype=np.uint8).copy()
    host_b = host_a.copy()
    L = libhv_amd.lib()
    L.hvws_set_validation(eng.ctx, 0)
    eng.rx_batch(host_a, [(0, len(data))], None, True)
    fa = eng.frames()
    L.hvws_set_validation(eng.ctx, V.V_ALL)
    eng.rx_batch(host_b, [(0, len(data))], None, True)
    fb = eng.frames()
    assert (host_a == host_b).all()                      # same bytes either way
    mask = ~np.uint32(I_INVALID | (63 << 16))
    assert (fa["info"] == (fb["info"] & mask)).all()     # only the validation bits differ
    for k in ("hdr_off", "pay_off", "pay_len", "length", "key"):
        assert (fa[k] == fb[k]).all()


@pytest.mark.parametrize("seed", [5, 6])
def test_classes_split_across_batches(eng, path, seed):
    """Headers cut at every possible byte by chunked batches: the partial
    validation state rides in the carry."""
    data, exp = V.random_stream(seed, 120)
    rng = random.Random(seed)
    L = libhv_amd.lib()
    L.hvws_set_validation(eng.ctx, V.V_ALL)
    carry = [None]
    got = []
    at = 0
    while at < len(data):
        n = min(len(data) - at, rng.choice([1, 2, 3, 5, 7, 11, 64, 500]))
        host = np.frombuffer(data[at:at + n], dtype=np.uint8).copy()
        carry = eng.rx_batch(host, [(0, n)], carry, True)
        got += _hdr_classes(eng.frames())
        at += n
    assert got == exp


def test_classes_many_segments(eng, path):
    streams = [V.random_stream(100 + i, 40) for i in range(37)]
    blob, segs = b"", []
    for d, _ in streams:
        segs.append((len(blob), len(d)))
        blob += d
    L = libhv_amd.lib()
    L.hvws_set_validation(eng.ctx, V.V_ALL)
    host = np.frombuffer(blob, dtype=np.uint8).copy()
    eng.rx_batch(host, segs, None, True)
    fr = eng.frames()
    first, cnt = eng.segment_frames(len(segs))
    for s, (_, exp) in enumerate(streams):
        assert _hdr_classes(fr[int(first[s]):int(first[s] + cnt[s])]) == exp


def _valid_then_bad(seed):
    rng = random.Random(seed)
    parts = []
    while True:
        b, v = V.make_frame(rng, p_bad=0.15)
        if v:
            bad = b
            break
        parts.append(b)
    return b"".join(parts), bad, len(parts)


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_execute_rejects_like_failing_header_callback(path, seed):
    good, bad, k = _valid_then_bad(seed)
    data = good + bad + b"\x82\x00"
    L = libhv_amd.lib()
    L.hvws_set_validation(None, V.V_ALL)
    log, _ = H.run_evlog("gpu", data, [len(data)])
    ev = H.parse_log(log)
    r = next(i for i, e in enumerate(ev) if e[0] == "R")
    # the header of the first violating frame is not delivered ...
    assert sum(e[0] == "H" for e in ev[:r]) == k
    # ... and execute returns the index of its last header byte, as the
    # reference does when on_frame_header fails
    vio = V.violations(data)
    off = vio[k][0]
    b1 = data[off + 1]
    hlen = 2 + {126: 2, 127: 8}.get(b1 & 127, 0) + (4 if b1 & 128 else 0)
    assert ev[r][1] == off + hlen - 1
    # everything before it matches the reference (oracle) callback for callback
    olog, _ = H.run_evlog("oracle", good, [len(good)])
    oev = H.parse_log(olog)
    assert ev[:r] == oev[:len(oev) - 1]


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_feed_recv_data_rejects(path, seed):
    good, bad, k = _valid_then_bad(seed)
    data = good + bad
    L = libhv_amd.lib()
    L.hvws_set_validation(None, V.V_ALL)
    msgs, rets, _, _ = H.run_messages("gpu", data, [len(data)])
    omsgs, _, _, _ = H.run_messages("oracle", good, [len(good)])
    off = V.violations(data)[k][0]
    b1 = data[off + 1]
    hlen = 2 + {126: 2, 127: 8}.get(b1 & 127, 0) + (4 if b1 & 128 else 0)
    assert rets == [off + hlen - 1]
    assert msgs == omsgs


@pytest.mark.parametrize("seed", [31, 32, 33])
def test_feed_recv_data_rejected_chunk_bytes(path, seed):
    """What a caller may rely on in a chunk FeedRecvData rejected (DESIGN sec. 7,
    validation): the bytes before the violating header are exactly what the
    reference leaves there (the delivered frames' payloads unmasked), the
    violating header's own bytes are as received, and everything after it is
    either as received or unmasked with its frames' keys -- one or the other for
    the whole rest of the chunk (the GPU unmasks a read in one pass)."""
    good, bad, k = _valid_then_bad(seed)
    data = good + bad
    L = libhv_amd.lib()
    L.hvws_set_validation(None, V.V_ALL)
    _, rets, _, buf = H.run_messages("gpu", data, [len(data)])
    off = V.violations(data)[k][0]
    b1 = data[off + 1]
    hlen = 2 + {126: 2, 127: 8}.get(b1 & 127, 0) + (4 if b1 & 128 else 0)
    assert rets == [off + hlen - 1]
    _, _, _, obuf = H.run_messages("oracle", good, [len(good)])
    assert bytes(buf[:off]) == bytes(obuf[:off])
    assert bytes(buf[off:off + hlen]) == data[off:off + hlen]
    _, _, _, ubuf = H.run_messages("oracle", data, [len(data)])   # the reference validates nothing
    rest = bytes(buf[off + hlen:])
    assert rest in (data[off + hlen:], bytes(ubuf[off + hlen:]))


@pytest.mark.parametrize("feeder", [False, True], ids=["many", "feeder"])
def test_batched_feed_rejects(path, feeder):
    """hvws_feed_many and a feeder (whose worker context takes the creating
    thread's validation classes) reject each connection's first violating
    header exactly as that connection's own FeedRecvData does."""
    L = libhv_amd.lib()
    L.hvws_set_validation(None, V.V_ALL)
    cases = []
    for seed in (21, 22, 23, 24):
        good, bad, _ = _valid_then_bad(seed)
        cases.append(good + bad)
    cases.append(_valid_then_bad(25)[0])   # a connection with no violation
    exp = [H.run_messages("gpu", d, [len(d)])[:2] for d in cases]
    n = len(cases)
    sinks = [H.MsgLog() for _ in cases]
    cbs = [libhv_amd.MSG_CB(s._on) for s in sinks]
    hs = [L.hvws_wsp_new() for _ in cases]
    for h, cb in zip(hs, cbs):
        L.hvws_wsp_set_sink(h, cb, None)
    bufs = [ctypes.create_string_buffer(d, len(d)) for d in cases]
    hv = (ctypes.c_void_p * n)(*hs)
    ds = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])
    ls = (ctypes.c_size_t * n)(*[len(d) for d in cases])
    rets = (ctypes.c_int * n)()
    if feeder:
        f = L.hvws_feeder_new()
        assert L.hvws_wsp_feeder_submit(f, hv, ds, ls, n, rets) == n
        L.hvws_feeder_free(f)
    else:
        assert L.hvws_wsp_feed_many(hv, ds, ls, n, rets) == n
    for i in range(n):
        assert (sinks[i].msgs, [rets[i]]) == exp[i], i
        L.hvws_wsp_free(hs[i])
