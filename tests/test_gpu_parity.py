"""GPU parity: the product (libhv_amd/libhvws.so, HIP kernels on MI355X)
against the CPU oracle on the same seeded inputs.  Integer/byte work, so the
bar is bit-exact everywhere."""
from __future__ import annotations

import ctypes
import random

import numpy as np
import pytest

import libhv_amd
import streams as S
import wsharness as H
from libhv_amd import synth

pytestmark = pytest.mark.gpu

@pytest.fixture(params=["small", "general"], autouse=True)
def rx_path(request):
    """Run every case through both host-batch paths: the single-launch
    small-batch kernel (default for reads this size) and the general
    COUNT/EMIT/unmask sequence.  Results must be identical."""
    L = libhv_amd.lib()
    limit = 0 if request.param == "small" else (1 << 64) - 1
    L.hvws_set_small_batch_limit(None, limit)
    eng = request.getfixturevalue("eng") if "eng" in request.fixturenames else None
    if eng:
        L.hvws_set_small_batch_limit(eng.ctx, limit)
    yield request.param
    L.hvws_set_small_batch_limit(None, 0)
    if eng:
        L.hvws_set_small_batch_limit(eng.ctx, 0)


@pytest.fixture(params=[256, 0], ids=["verify256", "verify_default"])
def spec_min(request):
    """Grid-wide uniform-run verification (k_verify) from 256 predicted frames
    (so these small cases exercise it) and at the default threshold (where
    k_walk's wave speculation verifies them)."""
    L = libhv_amd.lib()
    old = L.hvws_set_spec_min(request.param)
    yield request.param
    L.hvws_set_spec_min(old)


# ------------------------------------------------ reference frame-layer ABI
@pytest.mark.parametrize("name,data", S.quirk_streams(), ids=[n for n, _ in S.quirk_streams()])
@pytest.mark.parametrize("mode", ["one", "bytes", "small"])
@pytest.mark.parametrize("decode", [False, True])
def test_execute_quirks(name, data, mode, decode):
    rng = random.Random(hash((name, mode)) & 0xFFFF)
    if mode == "bytes" and len(data) > 400:
        mode = "small"
    chunks = S.rand_chunks(rng, len(data), mode)
    assert H.run_evlog("gpu", data, chunks, -1, decode) == H.run_evlog("oracle", data, chunks, -1, decode)


def test_execute_random_streams():
    rng = random.Random(1234)
    for t in range(60):
        data = S.rand_stream(rng, rng.randint(1, 10), max_len=rng.choice([40, 300, 3000]))
        mode = "small" if len(data) > 600 else None
        chunks = S.rand_chunks(rng, len(data), mode)
        decode = rng.random() < 0.5
        got = H.run_evlog("gpu", data, chunks, -1, decode)
        exp = H.run_evlog("oracle", data, chunks, -1, decode)
        assert got == exp, f"stream {t}"


def test_execute_early_return():
    """A callback returning non-zero stops the parse at the reference's cursor
    (http/websocket_parser.c:14-32); the caller re-feeds from there."""
    rng = random.Random(77)
    for t in range(40):
        data = S.rand_stream(rng, rng.randint(2, 6), max_len=200)
        chunks = S.rand_chunks(rng, len(data), "rand")
        abort_at = rng.randint(0, 12)
        decode = rng.random() < 0.5
        assert H.run_evlog("gpu", data, chunks, abort_at, decode) == \
            H.run_evlog("oracle", data, chunks, abort_at, decode), f"stream {t} abort {abort_at}"


def test_decode_helpers():
    L = libhv_amd.lib()
    O = H.oracle()
    rng = random.Random(5)
    for n in [0, 1, 3, 4, 15, 16, 17, 1000, 65536 + 7]:
        src = rng.randbytes(n)
        key = rng.randbytes(4)
        for ph in range(6):
            a = ctypes.create_string_buffer(max(n, 1))
            b = ctypes.create_string_buffer(max(n, 1))
            ra = L.websocket_decode(a, src, n, key, ph)
            rb = O.ows_decode(b, src, n, key, ph)
            assert ra == rb and a.raw[:n] == b.raw[:n]


def test_build_frame_matches_reference_layout():
    L = libhv_amd.lib()
    rng = random.Random(9)
    for n in S.EDGE_LENS + [1000, 70000]:
        data = rng.randbytes(n)
        key = rng.randbytes(4)
        for fl in (0x1 | 0x10 | 0x20, 0x2 | 0x20, 0x9 | 0x10, 0x0):
            buf = ctypes.create_string_buffer(n + 16)
            m = L.websocket_build_frame(buf, fl, key, data, n)
            exp = H.build_frames_ref([(fl, data, key)])
            assert buf.raw[:m] == exp
            assert L.websocket_calc_frame_size(fl, n) == len(exp)


# ----------------------------------------------------- message layer drop-in
@pytest.mark.parametrize("name,data", S.quirk_streams(), ids=[n for n, _ in S.quirk_streams()])
def test_messages_quirks(name, data):
    for mode in ("one", "small"):
        chunks = S.rand_chunks(random.Random(3), len(data), mode)
        assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks)


def test_messages_known_answers():
    """SURVEY.md Appendix A, probed with the compiled reference."""
    q = dict(S.quirk_streams())
    msgs, _, _, buf = H.run_messages("gpu", q["q5_control_between_fragments"], [1 << 20])
    assert msgs == [(9, b"ABPING"), (9, b"CD")]
    msgs, _, _, _ = H.run_messages("gpu", q["q6_lone_continue"], [1 << 20])
    assert msgs == [(8, b"orphan")]
    msgs, _, _, buf = H.run_messages("gpu", q["q10_inplace"], [1 << 20])
    assert buf == bytes.fromhex("81851122334448656c6c6f") and msgs == [(1, b"Hello")]
    msgs, _, _, _ = H.run_messages("gpu", q["rfc_hello_masked"], [3, 3, 5])
    assert msgs == [(1, b"Hello")]


def _long_header_stream(length: int, body: int, seed: int) -> bytes:
    """A masked binary frame header announcing `length` payload bytes (the
    8-byte form), then only `body` of them (the message never completes)."""
    rng = random.Random(seed)
    key = rng.randbytes(4)
    return bytes([0x82, 0xFF]) + length.to_bytes(8, "big") + key + rng.randbytes(body)


# Q11 (http/WebSocketParser.cpp:15-16): the reference
# stores parser->length in an int before reserve(); lengths in [2^31, 2^32)
# mod 2^32 go negative, become a huge size_t and reserve() throws
# std::length_error out of the parse.  Here (and in the oracle,
# oracle/ws_msg.cpp:68-72) a negative value reserves nothing and the message
# accumulates: a deliberate deviation, so this case is
# "parity unpinned" -- pinned to the oracle's documented behaviour only.
Q11_LENGTHS = [(1 << 31) - 1, 1 << 31, (1 << 31) + 5, (1 << 32) - 1, (1 << 32) + 7, (1 << 63) - 1]


@pytest.mark.parametrize("length", Q11_LENGTHS)
def test_messages_q11_long_length_header(length):
    data = _long_header_stream(length, 3000, length & 0xFFFF)
    for mode in ("one", "small"):
        chunks = S.rand_chunks(random.Random(11), len(data), mode)
        got = H.run_messages("gpu", data, chunks)
        assert got == H.run_messages("oracle", data, chunks)
        msgs, rets, st, _ = got
        assert msgs == [] and sum(rets) == len(data)   # no throw, every byte consumed
        assert st[4] == length and st[5] == length - 3000   # body state: length, bytes still required


def test_messages_random_chunked():
    rng = random.Random(4321)
    for t in range(25):
        data = S.rand_stream(rng, rng.randint(1, 12), max_len=rng.choice([100, 5000, 70000]))
        chunks = S.rand_chunks(rng, len(data), "rand")
        assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks), f"stream {t}"


# ------------------------------------------------------------ batch engine
def _oracle_batch(buf: np.ndarray, segs, carries):
    exp = buf.copy()
    recs, outs, starts = [], [], []
    for i, (off, n) in enumerate(segs):
        r, st, started, out = H.scan_segment(buf[off:off + n].tobytes(), carries[i] if carries else None)
        r = r.copy()
        r["pay_off"] += np.uint64(off)
        r["hdr_off"] = np.where(r["hdr_off"] >= 0, r["hdr_off"] + off, -1)
        recs.append(r)
        outs.append(st)
        starts.append(started)
        exp[off:off + n] = np.frombuffer(out, np.uint8)
    return np.concatenate(recs) if recs else np.zeros(0, libhv_amd.FRAME_DTYPE), outs, starts, exp


# Scan paths a multi-segment batch can take (include/hvws.h HVWS_PATH_*):
# (fast-bound threshold, speculation mode).  The default sends these small
# batches COUNT -> EMIT with no wait; threshold 1 forces the large-batch
# path, without speculation (COUNT, read, EMIT) and with it (speculative
# EMIT checked on the device, exact re-scan when the check fails): SPEC
# (uniform estimates) and SLACK (per-segment regions, compacted).
# The one-walk passes (SPEC, SLACK) run adaptively (default), with the
# k_verify pair forced ("_verify", fourth field 1) and without it
# ("_noverify", 0: head + walk, the walk records the carried-in frame).
# The RUN path (fifth field 1: hvws_set_run forced) takes every multi-segment
# batch of a step, uniform or not: a segment that is not one run of equal
# frames fails its check in the unmask and is repaired exactly on the device,
# so these modes also run the repair pass on every mixed batch.
SCAN_MODES = [("default", 0, -1), ("count_read", 1, 0), ("speculate", 1, 1),
              ("speculate_verify", 1, 1, 1), ("speculate_noverify", 1, 1, 0),
              ("pipelined", 0, -1), ("pipelined_speculate", 1, 1),
              ("slack", 1, 2), ("slack_noverify", 1, 2, 0), ("pipelined_slack", 1, 2),
              ("pipelined_slack_verify", 1, 2, 1), ("run", 1, 1, -1, 1), ("pipelined_run", 1, 1, -1, 1)]


def _step_checked(eng, buf, segs, carries, exp_recs, exp_carry, exp_started, exp, mode):
    L = libhv_amd.lib()
    bound, spec = mode[1], mode[2]
    verify = mode[3] if len(mode) > 3 else -1
    run = mode[4] if len(mode) > 4 else 0   # RUN only where a mode asks for it (test_gpu_run.py: automatic)
    old_b = L.hvws_set_fast_bound(eng.ctx, bound)
    old_s = L.hvws_set_speculation(eng.ctx, spec)
    old_v = L.hvws_set_walk_verify(eng.ctx, verify)
    old_r = L.hvws_set_run(eng.ctx, run)
    try:
        rx = eng.to_device(buf)
        if mode[0].startswith("pipelined"):
            eng.step_resident(rx, len(buf), segs, carries)
        else:
            eng.step(rx, len(buf), segs, carries)
        got = rx.download(len(buf))
        frames = eng.frames()
        cout, started = eng.carry(len(segs))
        rx.free()
        path = L.hvws_last_scan_path(eng.ctx)
    finally:
        L.hvws_set_fast_bound(eng.ctx, 0 if old_b == 1 << 24 else old_b)
        L.hvws_set_speculation(eng.ctx, old_s)
        L.hvws_set_walk_verify(eng.ctx, old_v)
        L.hvws_set_run(eng.ctx, old_r)
    if run == 1 and len(segs) > 1:
        assert path == 7, (mode, path)   # HVWS_PATH_RUN
    assert len(frames) == len(exp_recs), mode
    for f in ("hdr_off", "pay_off", "pay_len", "length", "key", "info"):
        assert np.array_equal(frames[f], exp_recs[f]), (mode, f)
    assert np.array_equal(got, exp), mode
    for s in range(len(segs)):
        assert cout[s].fields() == exp_carry[s].fields(), (mode, s)
        assert started[s] == exp_started[s], (mode, s)
    return path


def _compare_batch(eng, buf: np.ndarray, segs, carries=None):
    """The batch through every scan path, each bit-exact against the oracle.
    Returns {mode name: HVWS_PATH_* taken}."""
    exp_recs, exp_carry, exp_started, exp = _oracle_batch(buf, segs, carries)
    return {m[0]: _step_checked(eng, buf, segs, carries, exp_recs, exp_carry, exp_started, exp, m)
            for m in SCAN_MODES}


def test_batch_segments_with_carry(eng):
    """Many connections in one batch, each continuing mid-stream (cut at
    arbitrary bytes, including inside headers) from its carried parser state."""
    rng = random.Random(99)
    for trial in range(6):
        parts, segs, carries = [], [], []
        at = 0
        for c in range(rng.randint(1, 40)):
            data = S.rand_stream(rng, rng.randint(1, 20), max_len=rng.choice([50, 400, 70000]))
            a = rng.randint(0, len(data))
            b = rng.randint(a, len(data))
            # carry-in = oracle state after [0, a)
            _, st, _, _ = H.scan_segment(data[:a])
            gap = rng.choice([0, 0, 3, 16])
            parts.append(bytes(gap))
            at += gap
            parts.append(data[a:b])
            segs.append((at, b - a))
            carries.append(st)
            at += b - a
        buf = np.frombuffer(b"".join(parts), np.uint8).copy()
        _compare_batch(eng, buf, segs, carries)


def test_batch_every_cut_point(eng):
    """One frame of each header size cut at every byte: segment 1 ends there,
    segment 2 (same connection, next batch) resumes from its carry."""
    k = b"\x01\x02\x03\x04"
    for L in (5, 300, 70000):
        data = H.build_frames_ref([(2 | 0x10 | 0x20, bytes(range(256)) * (L // 256) + bytes(L % 256), k),
                                   (1 | 0x10 | 0x20, b"tail", k)])
        cuts = list(range(0, 20)) + [len(data) // 2, len(data) - 5, len(data) - 1, len(data)]
        for cut in cuts:
            _compare_batch(eng, np.frombuffer(data[:cut], np.uint8).copy(), [(0, cut)])
            _, st, _, _ = H.scan_segment(data[:cut])
            rest = np.frombuffer(data[cut:], np.uint8).copy()
            _compare_batch(eng, rest, [(0, len(rest))], [st])


def test_batch_empty_and_tiny(eng):
    _compare_batch(eng, np.zeros(0, np.uint8), [(0, 0)])
    _compare_batch(eng, np.frombuffer(bytes([0x82]), np.uint8).copy(), [(0, 1)])
    _compare_batch(eng, np.frombuffer(bytes([0x82, 0x80]), np.uint8).copy(), [(0, 2)])
    _compare_batch(eng, np.frombuffer(bytes([0x82, 0x00, 0x82, 0x00]), np.uint8).copy(), [(0, 2), (2, 2)])


def test_synth_matches_oracle(eng):
    for plan in (synth.uniform_plan(300, 1024, 5, opcode=1, text=True),
                 synth.uniform_plan(20, 70000, 6),
                 synth.mixed_plan(8 << 20, 7, hi=1 << 19)):
        host = H.synth_cpu(plan)
        dp = libhv_amd.DevicePlan(eng, plan)
        rx = eng.alloc(plan.total + 64)
        eng.synth(rx, plan.total, plan.seed, dp, 0)
        assert np.array_equal(rx.download(plan.total), host)
        assert eng.synth(rx, plan.total, plan.seed, dp, 1) == 0
        assert eng.digest(rx, plan.total) == H.digest_np(host)
        dp.free()
        rx.free()


@pytest.mark.parametrize("nseg", [1, 7, 256])
@pytest.mark.parametrize("kind", ["u1k", "u64k", "mixed"])
def test_batch_configs_small(eng, spec_min, kind, nseg):
    plan = {"u1k": lambda: synth.uniform_plan(4000, 1024, 11),
            "u64k": lambda: synth.uniform_plan(300, 65536, 12),
            "mixed": lambda: synth.mixed_plan(24 << 20, 13)}[kind]().split(nseg)
    host = H.synth_cpu(plan)
    _compare_batch(eng, host, plan.segments)


def test_rx_batch_host_roundtrip(eng):
    plan = synth.mixed_plan(4 << 20, 21, hi=1 << 18).split(5)
    host = H.synth_cpu(plan)
    _, _, _, exp = _oracle_batch(host, plan.segments, None)
    buf = host.copy()
    eng.rx_batch(buf, plan.segments, None, True)
    assert np.array_equal(buf, exp)


@pytest.mark.parametrize("payload,unmask", [(10, True), (10, False), (0, True), (0, False)],
                         ids=["512rec_unmask", "512rec_raw", "1365rec_unmask", "1365rec_raw"])
def test_rx_batch_small_path_over_host_record_area(eng, payload, unmask):
    """A small-path batch (k_small) with more records than the pinned record
    area holds (2^20): segments past it hand their records back through their
    device slots, which must be complete -- also for segments of <= 512
    records (kept in LDS) and without the unmask.  8 KiB segments of 16-byte
    frames (512 records each) or 6-byte empty frames (1365 each)."""
    n_seg = 4096 if payload else 1024
    per = 8192 // (payload + 6)
    plan = synth.uniform_plan(n_seg * per, payload, 23)
    plan.segments = [(s * per * (payload + 6), per * (payload + 6)) for s in range(n_seg)]
    host = H.synth_cpu(plan)
    exp_recs, exp_carry, _, exp = _oracle_batch(host, plan.segments, None)
    assert len(exp_recs) > 1 << 20
    libhv_amd.lib().hvws_set_small_batch_limit(eng.ctx, 0)   # default: batches <= 64 MiB take k_small
    buf = host.copy()
    eng.rx_batch(buf, plan.segments, None, unmask)
    assert np.array_equal(buf, exp if unmask else host)
    frames = eng.frames()
    assert len(frames) == len(exp_recs)
    for f in ("hdr_off", "pay_off", "pay_len", "length", "key", "info"):
        assert np.array_equal(frames[f], exp_recs[f]), f


def test_pipeline_host_inclusive(eng):
    """Chunked H2D -> scan -> unmask -> D2H with the carry chained across chunk
    boundaries (frames straddle chunks)."""
    plan = synth.mixed_plan(12 << 20, 31, hi=1 << 19)
    host = H.synth_cpu(plan)
    _, _, _, exp = _oracle_batch(host, [(0, plan.total)], None)
    L = libhv_amd.lib()
    pinned = L.hvws_host_alloc(eng.ctx, plan.total)
    try:
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * plan.total).from_address(pinned))
        arr[:] = host
        carry = libhv_amd.WsParser()
        L.websocket_parser_init(ctypes.byref(carry))
        rc = L.hvws_pipeline(eng.ctx, pinned, plan.total, 1 << 20, ctypes.byref(carry))
        assert rc == 0, L.hvws_last_error()
        assert np.array_equal(arr, exp)
        assert carry.state == 0
    finally:
        L.hvws_host_free(eng.ctx, pinned)


def test_stream_xor_roundtrip(eng):
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    b = eng.to_device(a)
    eng.stream_xor(b, len(a), 0xA5A5A5A5)
    x = b.download(len(a))
    assert np.array_equal(x, a ^ np.uint8(0xA5))
    b.free()


def test_batch_dense_tiny_frames(eng, spec_min):
    """Many frames inside one 16-byte chunk (2-byte unmasked empties between
    masked ones) at every alignment: the unmask kernel's boundary merge must
    visit each payload piece."""
    rng = random.Random(2024)
    k = b"\x9a\x5c\x33\xe1"
    for pad in range(16):
        frames = []
        for _ in range(400):
            r = rng.random()
            if r < 0.4:
                frames.append((0x2 | 0x10, b"", None))                      # 2-byte unmasked empty
            elif r < 0.6:
                frames.append((0x2 | 0x10 | 0x20, b"", k))                  # 6-byte masked empty
            else:
                frames.append((0x1 | 0x10 | 0x20, rng.randbytes(rng.randint(1, 20)), rng.randbytes(4)))
        data = bytes(pad) + H.build_frames_ref(frames)
        buf = np.frombuffer(data, np.uint8).copy()
        _compare_batch(eng, buf, [(pad, len(data) - pad)])


def test_unmask_geometries(eng):
    """Every compiled k_unmask geometry (the engine picks one by batch size:
    include/hvws.h hvws_set_unmask_variant) on batches with every tile class:
    dense tiny frames (boundary chunks), mixed sizes with fragments and pings,
    64 KiB frames (single-payload tiles), unmasked frames (empty tiles) --
    bytes and frames bit-exact against the oracle."""
    L = libhv_amd.lib()
    rng = random.Random(4242)
    k = b"\x9a\x5c\x33\xe1"
    dense = [(0x2 | 0x10 | 0x20, rng.randbytes(rng.randint(0, 30)), rng.randbytes(4)) for _ in range(3000)]
    cases = [np.frombuffer(bytes(5) + H.build_frames_ref(dense), np.uint8).copy()]
    mplan = synth.mixed_plan(6 << 20, 4243, hi=1 << 18).split(13)
    cases.append(H.synth_cpu(mplan))
    uplan = synth.uniform_plan(40, 65536, 4244).split(3)
    cases.append(H.synth_cpu(uplan))
    plain = [(0x2 | 0x10, rng.randbytes(70000), None), (0x1 | 0x10 | 0x20, rng.randbytes(50000), k)] * 4
    cases.append(np.frombuffer(H.build_frames_ref(plain), np.uint8).copy())
    segss = [[(5, len(cases[0]) - 5)], mplan.segments, uplan.segments, [(0, len(cases[3]))]]
    nvar = 0
    while L.hvws_set_unmask_variant(nvar) == 0:
        nvar += 1
    assert nvar == 2, nvar   # 256 x 4 XCD-ordered, 512 x 2 linear (round 6 removed the rest)
    try:
        for buf, segs in zip(cases, segss):
            exp_recs, _, _, exp = _oracle_batch(buf, segs, None)
            for v in range(nvar):
                assert L.hvws_set_unmask_variant(v) == 0
                rx = eng.to_device(buf)
                eng.step(rx, len(buf), segs, None)
                got = rx.download(len(buf))
                frames = eng.frames()
                rx.free()
                name = L.hvws_unmask_kernel_name().decode()
                assert np.array_equal(got, exp), name
                assert len(frames) == len(exp_recs), name
                for f in ("hdr_off", "pay_off", "pay_len", "length", "key", "info"):
                    assert np.array_equal(frames[f], exp_recs[f]), (name, f)
    finally:
        L.hvws_set_unmask_variant(-1)
    # by size: small batches run the linear geometry, 16 GiB and up the XCD-contiguous one
    assert L.hvws_unmask_kernel_name_for(1 << 30).decode() == "k_unmask<512,2,linear>"
    assert L.hvws_unmask_kernel_name_for(64 << 30).decode() == "k_unmask<256,4,xcd>"


def test_long_segment_speculation_breaks(eng, spec_min):
    """Uniform runs verified in parallel, broken by a different size at many
    positions (the prefix verifier must stop exactly at the first break)."""
    rng = random.Random(31)
    for brk in (1, 2, 255, 256, 257, 300, 511, 1000):
        frames = [(0x2 | 0x10 | 0x20, rng.randbytes(100), rng.randbytes(4)) for _ in range(1200)]
        frames[brk] = (0x2 | 0x20, rng.randbytes(101), rng.randbytes(4))   # one odd size, FIN=0
        if brk + 5 < len(frames):
            frames[brk + 5] = (0x0 | 0x10, rng.randbytes(104), None)       # unmasked, same stride
        data = H.build_frames_ref(frames)
        cut = len(data) - rng.randint(0, 150)
        buf = np.frombuffer(data[:cut], np.uint8).copy()
        _compare_batch(eng, buf, [(0, cut)])
        _, st, _, _ = H.scan_segment(data[:cut])
        rest = np.frombuffer(data[cut:], np.uint8).copy()
        _compare_batch(eng, rest, [(0, len(rest))], [st])


def test_long_segment_last_frame_unmasked(eng, spec_min):
    """Verified prefix ending in an unmasked frame of the same stride: the
    carried mask must be the last *masked* key (Q14, stale mask)."""
    rng = random.Random(41)
    for n_frames in (256, 257, 700):
        frames = [(0x2 | 0x10 | 0x20, rng.randbytes(100), rng.randbytes(4)) for _ in range(n_frames)]
        frames[-1] = (0x2 | 0x10, rng.randbytes(104), None)
        frames[-2] = (0x2 | 0x10, rng.randbytes(104), None)
        data = H.build_frames_ref(frames)
        _compare_batch(eng, np.frombuffer(data, np.uint8).copy(), [(0, len(data))])
        # and with a partial header of a next frame after it
        data2 = data + H.build_frames_ref([(0x1 | 0x20, b"abc", b"wxyz")])[:4]
        _compare_batch(eng, np.frombuffer(data2, np.uint8).copy(), [(0, len(data2))])


def _cut_uniform(rng, nframes, size, nseg, masked=True):
    """One uniform stream cut into nseg segments at random bytes (headers
    split across segments included); returns (buf, segs, carries)."""
    frames = [((0x2 | 0x10 | 0x20) if masked else (0x2 | 0x10), rng.randbytes(size), rng.randbytes(4) if masked else None)
              for _ in range(nframes)]
    data = H.build_frames_ref(frames)
    cuts = sorted(rng.sample(range(1, len(data)), nseg - 1))
    bounds = [0] + cuts + [len(data)]
    segs, carries = [], []
    for a, b in zip(bounds[:-1], bounds[1:]):
        _, st, _, _ = H.scan_segment(data[:a])
        segs.append((a, b - a))
        carries.append(st)
    return np.frombuffer(data, np.uint8).copy(), segs, carries


def test_speculative_table_uniform(eng):
    """Uniform streams cut anywhere: every segment's record count is what
    k_head estimates, so the speculative table passes the device check."""
    rng = random.Random(77)
    for size, nframes, nseg in ((1024, 900, 13), (100, 3000, 64), (70000, 40, 9), (0, 500, 5), (125, 700, 700)):
        buf, segs, carries = _cut_uniform(rng, nframes, size, nseg)
        paths = _compare_batch(eng, buf, segs, carries)
        assert paths["speculate"] == 3, paths   # HVWS_PATH_SPEC
        assert paths["count_read"] == 1, paths


def test_speculative_table_rejected(eng):
    """Mixed sizes: the estimates fail, the device zeroes the count (no tile
    or unmask work) and the host re-scans exactly -- same bytes and records."""
    plan = synth.mixed_plan(6 << 20, 17, hi=1 << 17).split(37)
    host = H.synth_cpu(plan)
    paths = _compare_batch(eng, host, plan.segments)
    assert paths["speculate"] == 4, paths       # HVWS_PATH_SPEC_FAILED


def test_speculation_adapts(eng):
    """Automatic mode: SPEC for uniform traffic, SLACK for mixed, switching by
    what the last batch's check saw; a SLACK region sized by a lighter batch
    fails once and is re-sized by the exact re-scan.  Results stay exact."""
    L = libhv_amd.lib()
    rng = random.Random(5)
    ubuf, usegs, ucarry = _cut_uniform(rng, 300, 1024, 11)          # ~27 records per segment
    mplan = synth.mixed_plan(4 << 20, 19, hi=1 << 14).split(11)     # >100 records per segment
    mbuf = H.synth_cpu(mplan)
    uexp = _oracle_batch(ubuf, usegs, ucarry)
    mexp = _oracle_batch(mbuf, mplan.segments, None)
    assert max(np.bincount(np.searchsorted(np.array([o for o, _ in mplan.segments]), mexp[0]["hdr_off"].clip(0),
                                           side="right") - 1)) > 1.5 * 28 + 16
    auto = ("auto", 1, -1)
    # reset (exact, mixed) -> ubuf: SLACK (sees uniform) -> ubuf: SPEC -> mbuf:
    # SPEC fails, SLACK (regions sized by ubuf) fails -> mbuf: SLACK -> ubuf:
    # SLACK (uniform again) -> ubuf: SPEC
    seq = [(ubuf, usegs, ucarry, uexp, 5), (ubuf, usegs, ucarry, uexp, 3), (mbuf, mplan.segments, None, mexp, 6),
           (mbuf, mplan.segments, None, mexp, 5), (ubuf, usegs, ucarry, uexp, 5), (ubuf, usegs, ucarry, uexp, 3)]
    L.hvws_set_speculation(eng.ctx, 0)   # forget what earlier tests taught the context
    _step_checked(eng, mbuf, mplan.segments, None, *mexp, ("reset", 1, 0))
    for i, (buf, segs, carries, exp, want) in enumerate(seq):
        path = _step_checked(eng, buf, segs, carries, *exp, auto)
        assert path == want, (i, path, want)


def test_pipelined_steps_back_to_back(eng):
    """hvws_step_resident on several resident batches with no wait between
    calls: each batch's discovery runs on the second stream while the
    previous batch is unmasked; every buffer must come out exact, and the
    last step's frames and carry must be its own."""
    L = libhv_amd.lib()
    rng = random.Random(123)
    batches = []
    for i in range(8):
        if i % 3 == 2:
            plan = synth.mixed_plan(3 << 20, 40 + i, hi=1 << 16).split(9)
            buf, segs, carries = H.synth_cpu(plan), plan.segments, None
        else:
            buf, segs, carries = _cut_uniform(rng, 400 + 50 * i, rng.choice([100, 1024, 3000]), 7 + i)
        batches.append((buf, segs, carries))
    for bound, spec in ((0, -1), (1, 1), (1, -1)):
        old_b = L.hvws_set_fast_bound(eng.ctx, bound)
        old_s = L.hvws_set_speculation(eng.ctx, spec)
        try:
            devs = [eng.to_device(b) for b, _, _ in batches]
            for d, (b, segs, carries) in zip(devs, batches):
                eng.step_resident(d, len(b), segs, carries)
            # a second pass over the first buffer restores its masked bytes
            # (its bytes must be complete first: the API's precondition)
            eng.sync()
            eng.step_resident(devs[0], len(batches[0][0]), batches[0][1], batches[0][2])
            frames = eng.frames()
            cout, started = eng.carry(len(batches[0][1]))
            got = [d.download(len(b)) for d, (b, _, _) in zip(devs, batches)]
            for d in devs:
                d.free()
        finally:
            L.hvws_set_fast_bound(eng.ctx, 0 if old_b == 1 << 24 else old_b)
            L.hvws_set_speculation(eng.ctx, old_s)
        assert np.array_equal(got[0], batches[0][0]), (bound, spec)
        for i in range(1, len(batches)):
            b, segs, carries = batches[i]
            assert np.array_equal(got[i], _oracle_batch(b, segs, carries)[3]), (bound, spec, i)
        # the last call scanned batch 0 in its unmasked state: its frames are
        # those of the unmasked bytes
        b0, segs0, carries0 = batches[0]
        unm = _oracle_batch(b0, segs0, carries0)[3]
        exp_recs, exp_carry, _, _ = _oracle_batch(unm, segs0, carries0)
        assert len(frames) == len(exp_recs)
        for f in ("hdr_off", "pay_off", "pay_len", "length", "key", "info"):
            assert np.array_equal(frames[f], exp_recs[f]), f
        for k in range(len(segs0)):
            assert cout[k].fields() == exp_carry[k].fields(), k


def test_step_event_interval(eng):
    """hvws_set_step_event_interval: pipelined steps carry their timing events
    on every n-th scan only (unsampled steps read -1; 0 = none), and the bytes
    do not depend on it (12 passes: the batch is masked again)."""
    rng = random.Random(77)
    buf, segs, carries = _cut_uniform(rng, 3000, 1024, 16)
    d = eng.to_device(buf)
    try:
        for every, want in ((3, 4), (0, 0), (1, 12)):
            assert eng.set_step_event_interval(every) >= 0
            for _ in range(12):
                eng.step_resident(d, len(buf), segs, carries)
            eng.sync()
            times = eng.step_times(12)
            got = [i for i, (_, u) in enumerate(times) if u >= 0]
            assert len(times) == 12 and len(got) == want, (every, times)
            assert all(times[i][1] > 0 for i in got)
            if every > 1:
                assert all(b - a == every for a, b in zip(got, got[1:])), got
            assert np.array_equal(d.download(len(buf)), buf), every
    finally:
        eng.set_step_event_interval(1)
        d.free()


def _piped_after_stall(eng, learn, target, spec_learn, spec_target, bound=1, stall_us=150_000):
    """Pipelined step of `learn`, then a host stall on the context stream (a
    stand-in for a long previous unmask: everything queued there after it
    waits), then a pipelined step of `target` whose check is rejected.
    The pair runs twice and the second is checked: the first sizes the
    target's table set, so the re-scan reallocates nothing (a reallocation's
    hipFree would synchronise the device and hide the race).
    Returns (target bytes after its step, target frames, target's path)."""
    L = libhv_amd.lib()
    old_b = L.hvws_set_fast_bound(eng.ctx, bound)
    try:
        lbuf, lsegs = learn
        tbuf, tsegs = target
        for rep in range(2):
            L.hvws_set_speculation(eng.ctx, spec_learn)
            dl, dt = eng.to_device(lbuf), eng.to_device(tbuf)
            eng.step_resident(dl, len(lbuf), lsegs, None)
            L.hvws_set_speculation(eng.ctx, spec_target)
            if rep:
                libhv_amd._check(L.hvws_debug_stall(eng.ctx, stall_us), "hvws_debug_stall")
            eng.step_resident(dt, len(tbuf), tsegs, None)
            path = L.hvws_last_scan_path(eng.ctx)
            eng.sync()
            got = dt.download(len(tbuf))
            frames = eng.frames()
            dl.free()
            dt.free()
    finally:
        L.hvws_set_fast_bound(eng.ctx, 0 if old_b == 1 << 24 else old_b)
        L.hvws_set_speculation(eng.ctx, -1)
    return got, frames, path


def test_pipelined_rejected_check_waits_for_queued_unmask():
    """A pipelined step whose speculative check is rejected (SPEC, SLACK, or a
    one-stream table that overflowed its estimate) has already queued its
    speculative unmask on the context stream, behind the previous batch's
    unmask.  The exact re-scan runs on the second stream and rewrites the same
    tile index: it must wait for that unmask, or the unmask (running late)
    sees the new tiles and XORs for real and the caller's unmask XORs the
    payloads back.  A host stall on the context stream holds the queued unmask
    back for 150 ms so the window is certain to be open."""
    rng = random.Random(606)
    lplan = synth.uniform_plan(600, 1024, 608).split(9)   # uniform traffic first
    lbuf = H.synth_cpu(lplan)
    mplan = synth.mixed_plan(4 << 20, 607, hi=1 << 15).split(9)
    mbuf = H.synth_cpu(mplan)
    mexp_recs, _, _, mexp = _oracle_batch(mbuf, mplan.segments, None)

    def check(got, frames, path, want_path, exp, exp_recs):
        assert path == want_path, path
        assert np.array_equal(got, exp)
        assert len(frames) == len(exp_recs)
        for f in ("hdr_off", "pay_off", "pay_len", "length", "key", "info"):
            assert np.array_equal(frames[f], exp_recs[f]), f

    # SPEC rejected (mixed target after uniform traffic, SPEC forced)
    with libhv_amd.Engine(0) as fresh:
        got, frames, path = _piped_after_stall(fresh, (lbuf, lplan.segments), (mbuf, mplan.segments), 1, 1)
        check(got, frames, path, 4, mexp, mexp_recs)   # HVWS_PATH_SPEC_FAILED

    # SLACK rejected: regions sized by a light batch, a dense one outgrows them
    small = synth.mixed_plan(3 << 20, 609, lo=1000, hi=1 << 16).split(29)
    sbuf = H.synth_cpu(small)
    dense = synth.mixed_plan(3 << 20, 610, lo=1, hi=300).split(5)
    dbuf = H.synth_cpu(dense)
    drecs, _, _, dexp = _oracle_batch(dbuf, dense.segments, None)
    with libhv_amd.Engine(0) as fresh:
        got, frames, path = _piped_after_stall(fresh, (sbuf, small.segments), (dbuf, dense.segments), 0, 2)
        check(got, frames, path, 6, dexp, drecs)       # HVWS_PATH_SLACK_FAILED

    # one stream whose table overflowed the first estimate (2^20 records)
    k = b"\x11\x22\x33\x44"
    frames_in = []
    for _ in range(1_100_000):
        if rng.random() < 0.8:
            frames_in.append((0x2 | 0x10, b"", None))
        else:
            frames_in.append((0x1 | 0x10 | 0x20, rng.randbytes(rng.randint(1, 9)), k))
    obuf = np.frombuffer(H.build_frames_ref(frames_in), np.uint8).copy()
    orecs, _, _, oexp = _oracle_batch(obuf, [(0, len(obuf))], None)
    # learn: one stream of 64 KiB frames whose record bound exceeds the table
    # guess, so its count is read and the next guess is back to 2^20
    splan = synth.uniform_plan(64, 65536, 611)
    sl = H.synth_cpu(splan)
    with libhv_amd.Engine(0) as fresh:
        got, frames, path = _piped_after_stall(fresh, (sl, [(0, len(sl))]), (obuf, [(0, len(obuf))]), -1, -1)
        check(got, frames, path, 2, oexp, orecs)       # HVWS_PATH_SINGLE (re-emitted)


def test_single_segment_table_overflow():
    """One segment with more records than the first one-stream table guess
    (2^20): the pass overflows, the count is read, the segment is re-emitted
    into an exact table; the next batch on the context is sized from it."""
    rng = random.Random(8)
    k = b"\x11\x22\x33\x44"
    frames = []
    for _ in range(1_200_000):
        if rng.random() < 0.8:
            frames.append((0x2 | 0x10, b"", None))                         # 2-byte unmasked empty
        else:
            frames.append((0x1 | 0x10 | 0x20, rng.randbytes(rng.randint(0, 9)), k))
    data = H.build_frames_ref(frames)
    buf = np.frombuffer(data, np.uint8).copy()
    with libhv_amd.Engine(0) as fresh:
        paths = _compare_batch(fresh, buf, [(0, len(buf))])
        assert set(paths.values()) == {2}, paths   # HVWS_PATH_SINGLE
        _compare_batch(fresh, buf[:len(buf) // 2].copy(), [(0, len(buf) // 2)])


# ------------------------------------------------------------ frame sieve
@pytest.fixture
def sieve_low():
    """Sieve one-segment batches from 4 KiB after their first whole frame
    (default 8 MiB) so these cases exercise it."""
    L = libhv_amd.lib()
    old = L.hvws_set_sieve_min(4096)
    yield
    L.hvws_set_sieve_min(old)


def _last_sieve(eng):
    out = (ctypes.c_uint64 * 4)()
    assert libhv_amd.lib().hvws_last_sieve(eng.ctx, out) == 0
    return list(out)


@pytest.mark.parametrize("target,lo,hi,seed", [(24 << 20, 128, 1 << 20, 51), (3 << 20, 1, 4096, 52),
                                               (1 << 20, 1, 200, 53), (12 << 20, 100, 70000, 54)])
def test_sieve_mixed_stream(eng, sieve_low, target, lo, hi, seed):
    """Config-4-shaped streams (fragments, pings, every length encoding) as
    one segment: the sieve's chain covers every frame, records and bytes
    bit-exact through every scan path."""
    plan = synth.mixed_plan(target, seed, lo=lo, hi=hi)
    host = H.synth_cpu(plan)
    paths = _compare_batch(eng, host, [(0, plan.total)])
    assert set(paths.values()) == {2}, paths   # HVWS_PATH_SINGLE
    active, surv, npath, pend = _last_sieve(eng)
    assert active == 1 and npath == plan.n and pend == plan.total, (active, surv, npath, pend, plan.n)
    rt, wt = _last_windows(eng)
    # every tile sieved: every frame is a survivor; windows: only theirs
    assert surv >= plan.n if rt == wt else 0 < surv, (surv, plan.n, rt, wt)


@pytest.fixture
def sieve_windows():
    """Set the sieve's window geometry for one test (hops, window bytes)."""
    L = libhv_amd.lib()
    prev = (ctypes.c_uint64 * 2)()
    L.hvws_set_sieve_windows(256, 0, prev)
    yield lambda hops, win: L.hvws_set_sieve_windows(hops, win, None)
    L.hvws_set_sieve_windows(prev[0], prev[1], None)


def _last_windows(eng):
    out = (ctypes.c_uint64 * 2)()
    assert libhv_amd.lib().hvws_last_sieve_windows(eng.ctx, out) == 0
    return list(out)


@pytest.mark.parametrize("target,lo,hi,seed,hops,win", [
    (24 << 20, 128, 1 << 20, 151, 64, (1 << 20) + (16 << 10)),   # config-4 shape, default window
    (24 << 20, 128, 1 << 20, 152, 8, 64 << 10),                  # windows shorter than frames: walks cross them
    (6 << 20, 1, 4096, 153, 256, 32 << 10),                      # small frames, long walks
    (12 << 20, 100, 70000, 154, 32, 16 << 10)])
def test_sieve_windows(eng, sieve_low, sieve_windows, target, lo, hi, seed, hops, win):
    """Windowed sieve: only the first `win` bytes of every region of ~hops
    frames are sieved, link walks cross the rest.  The first scan has no count
    (every tile); later ones are windowed.  Records and bytes bit-exact in
    every scan path, the chain covers every frame."""
    sieve_windows(hops, win)
    plan = synth.mixed_plan(target, seed, lo=lo, hi=hi)
    host = H.synth_cpu(plan)
    for _ in range(2):
        paths = _compare_batch(eng, host, [(0, plan.total)])
        assert set(paths.values()) == {2}, paths   # HVWS_PATH_SINGLE
    rt, wt = _last_windows(eng)
    assert wt > 0 and rt >= 2 * wt, (rt, wt)
    active, surv, npath, pend = _last_sieve(eng)
    assert active == 1 and npath == plan.n and pend == plan.total, (active, surv, npath, pend, plan.n)


def test_sieve_windows_walk_cap(eng, sieve_low, sieve_windows):
    """A region the link walks cannot cross within their frame cap (a run of
    tiny frames between large ones, one region for the whole stream): the
    chain stops, the exact walk finishes the segment (results exact), and the
    context sieves every tile for the next scans."""
    sieve_windows(1 << 20, 64 << 10)
    parts = [synth.mixed_plan(6 << 20, 161, lo=256 << 10, hi=1 << 20),
             synth.mixed_plan(1 << 20, 162, lo=1, hi=4),
             synth.mixed_plan(6 << 20, 163, lo=256 << 10, hi=1 << 20)]
    host = np.concatenate([H.synth_cpu(p) for p in parts])
    n = sum(p.n for p in parts)
    segs = [(0, len(host))]
    exp_recs, exp_carry, exp_started, exp = _oracle_batch(host, segs, None)
    assert len(exp_recs) == n
    kinds = []   # per scan: "full", "short" (windowed, chain stopped early) or "long"
    for i in range(20):
        mode = SCAN_MODES[i % 3]
        assert _step_checked(eng, host, segs, None, exp_recs, exp_carry, exp_started, exp, mode) == 2
        rt, wt = _last_windows(eng)
        active, _, npath, pend = _last_sieve(eng)
        assert active == 1
        kinds.append("full" if rt == wt else "short" if pend < len(host) else "long")
    # a windowed scan stops at the tiny frames; the scans after it sieve
    # every tile again
    assert "short" in kinds, kinds
    k = kinds.index("short")
    assert k + 1 < len(kinds) and kinds[k + 1] == "full", kinds


def test_sieve_cut_and_carried(eng, sieve_low):
    """A sieved stream cut at arbitrary bytes (inside headers, payloads, key
    bytes): the first batch ends with a partial frame, the second resumes
    from its carry -- both exact."""
    rng = random.Random(61)
    plan = synth.mixed_plan(2 << 20, 62, lo=1, hi=3000)
    data = H.synth_cpu(plan).tobytes()
    offs = [int(x) for x in plan.frame_off]
    for cut in [len(data) - 1, len(data) - 3, offs[-1] + 1, offs[-1] + 5, offs[-2] + 3, rng.randrange(len(data)),
                rng.randrange(len(data))]:
        _compare_batch(eng, np.frombuffer(data[:cut], np.uint8).copy(), [(0, cut)])
        _, st, _, _ = H.scan_segment(data[:cut])
        rest = np.frombuffer(data[cut:], np.uint8).copy()
        if len(rest):
            _compare_batch(eng, rest, [(0, len(rest))], [st])


def test_sieve_chain_breaks_on_quirks(eng, sieve_low):
    """Frames the plausibility filter rejects (unmasked, RSV bits, reserved
    opcodes, non-minimal lengths -- all accepted by the reference) inside a
    long mixed stream: the chain stops there and the exact walk takes over;
    results identical to the oracle."""
    rng = random.Random(71)
    base = H.synth_cpu(synth.mixed_plan(1 << 20, 72, lo=1, hi=5000)).tobytes()
    hdrs = [int(r) for r in H.scan_segment(base)[0]["hdr_off"]]
    k = b"\x0a\x0b\x0c\x0d"
    odd = [H.build_frames_ref([(0x2 | 0x10, rng.randbytes(300), None)]),                 # unmasked
           S.with_rsv(H.build_frames_ref([(0x1 | 0x10 | 0x20, rng.randbytes(40), k)])),   # RSV1
           H.build_frames_ref([(0x3 | 0x10 | 0x20, rng.randbytes(70), k)]),               # reserved opcode
           bytes([0x82, 0xFE, 0x00, 0x05]) + k + rng.randbytes(5)]                        # 16-bit length 5
    for pos_frac in (0.0, 0.3, 0.97):
        for o in odd:
            data = H.build_frames_ref([(0x1 | 0x10 | 0x20, b"first", k)])
            cut = int(len(base) * pos_frac)
            bnd = int(min((r for r in hdrs if r >= cut), default=len(base)))   # a frame boundary
            stream = data + base[:bnd] + o + base[bnd:]
            buf = np.frombuffer(stream, np.uint8).copy()
            _compare_batch(eng, buf, [(0, len(buf))])
            active, _, npath, pend = _last_sieve(eng)
            # the chain ends at or before the odd frame (a true frame survives
            # only if the 3 headers after it are plausible too)
            assert active == 1 and pend <= len(data) + bnd and (bnd < 20000 or npath > 0), (npath, pend, bnd)


def test_sieve_uniform_then_mixed(eng, sieve_low):
    """Uniform traffic leaves the sieve unwanted (the walk's stride
    speculation is exact and cheap); mixed traffic after it is sieved again
    once the context retries.  Results exact throughout."""
    rng = random.Random(81)
    ubuf, _, _ = _cut_uniform(rng, 3000, 1000, 1)
    mplan = synth.mixed_plan(2 << 20, 82, lo=1, hi=4000)
    mbuf = H.synth_cpu(mplan)
    _compare_batch(eng, ubuf, [(0, len(ubuf))])
    assert _last_sieve(eng)[0] == 0
    for _ in range(20):
        _compare_batch(eng, mbuf, [(0, len(mbuf))])
    assert _last_sieve(eng)[0] == 1


def test_sieve_survivor_overflow():
    """More survivors than the first table holds (2^20): the sieve stands
    down, the exact walk runs, and the next batch gets a table that fits."""
    rng = random.Random(91)
    k = b"\x21\x43\x65\x87"
    frames = [(0x2 | 0x10 | 0x20, rng.randbytes(rng.randint(0, 9)), k) for _ in range(1_100_000)]
    data = H.build_frames_ref(frames)
    buf = np.frombuffer(data, np.uint8).copy()
    L = libhv_amd.lib()
    old = L.hvws_set_sieve_min(4096)
    try:
        with libhv_amd.Engine(0) as fresh:
            _compare_batch(fresh, buf, [(0, len(buf))])
            st = _last_sieve(fresh)
            assert st[0] == 1 and st[2] == len(frames), st   # sized from the first pass's count
    finally:
        L.hvws_set_sieve_min(old)


def test_sieve_pipelined_same_buffer(eng, sieve_low):
    """bench.py's pattern: one resident one-segment batch stepped back to back
    with hvws_step_resident, so each step's discovery runs while the previous
    step still unmasks the same bytes.  Headers never change, so every step's
    records are the batch's; an even number of steps restores the bytes."""
    plan = synth.mixed_plan(16 << 20, 95, lo=1, hi=1 << 18)
    host = H.synth_cpu(plan)
    exp_recs, _, _, _ = _oracle_batch(host, [(0, plan.total)], None)
    rx = eng.to_device(host)
    for _ in range(6):
        eng.step_resident(rx, plan.total, [(0, plan.total)], None)
    eng.sync()
    frames = eng.frames()
    got = rx.download(plan.total)
    rx.free()
    assert np.array_equal(got, host)
    assert len(frames) == len(exp_recs)
    for f in ("hdr_off", "pay_off", "pay_len", "length", "key", "info"):
        assert np.array_equal(frames[f], exp_recs[f]), f
    assert _last_sieve(eng)[0] == 1


def test_sieve_pipeline_host_inclusive(eng, sieve_low):
    """hvws_pipeline over mixed traffic with every chunk sieved: frames straddle
    the 2 MiB chunks, each chunk's scan starts from the carried state."""
    plan = synth.mixed_plan(12 << 20, 97, hi=1 << 18)
    host = H.synth_cpu(plan)
    _, _, _, exp = _oracle_batch(host, [(0, plan.total)], None)
    L = libhv_amd.lib()
    pinned = L.hvws_host_alloc(eng.ctx, plan.total)
    try:
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * plan.total).from_address(pinned))
        arr[:] = host
        carry = libhv_amd.WsParser()
        L.websocket_parser_init(ctypes.byref(carry))
        rc = L.hvws_pipeline(eng.ctx, pinned, plan.total, 2 << 20, ctypes.byref(carry))
        assert rc == 0, L.hvws_last_error()
        assert np.array_equal(arr, exp)
        assert carry.state == 0
        assert _last_sieve(eng)[0] == 1
    finally:
        L.hvws_host_free(eng.ctx, pinned)


def test_slack_table_mixed_segments(eng):
    """Mixed sizes over many segments: one EMIT walk into per-segment regions,
    compacted on the device (HVWS_PATH_SLACK); a later batch whose segments
    outgrow their regions fails the check and is re-scanned exactly."""
    L = libhv_amd.lib()
    small = synth.mixed_plan(3 << 20, 101, lo=1000, hi=1 << 16).split(29)
    sbuf = H.synth_cpu(small)
    dense = synth.mixed_plan(3 << 20, 102, lo=1, hi=300).split(5)   # many more frames per segment
    dbuf = H.synth_cpu(dense)
    sexp = _oracle_batch(sbuf, small.segments, None)
    dexp = _oracle_batch(dbuf, dense.segments, None)
    L.hvws_set_speculation(eng.ctx, 0)
    _step_checked(eng, sbuf, small.segments, None, *sexp, ("exact", 1, 0))   # learns the region size
    assert _step_checked(eng, sbuf, small.segments, None, *sexp, ("slack", 1, 2)) == 5
    assert _step_checked(eng, dbuf, dense.segments, None, *dexp, ("slack", 1, 2)) == 6
    assert _step_checked(eng, dbuf, dense.segments, None, *dexp, ("slack", 1, 2)) == 5   # sized from the re-scan


def test_slack_carried_partial_frames_ends_monotone(eng):
    """SLACK over segments that each continue a frame carried in from an
    earlier batch (cut inside headers and payloads) and end inside one: the
    compacted table must equal the oracle's and its frame ends must never
    decrease -- the invariant k_tile_scatter / k_tile_fix_class rely on
    (every scan of the session also runs k_ends_check, conftest.py)."""
    L = libhv_amd.lib()
    assert L.hvws_set_table_checks(1) == 1
    rng = random.Random(707)
    parts, segs, carries = [], [], []
    at = 0
    for _ in range(23):
        data = S.rand_stream(rng, rng.randint(20, 60), max_len=rng.choice([300, 5000, 70000]))
        a = rng.randint(1, len(data) // 3)
        b = rng.randint(2 * len(data) // 3, len(data) - 1)
        _, st, _, _ = H.scan_segment(data[:a])
        parts.append(data[a:b])
        segs.append((at, b - a))
        carries.append(st)
        at += b - a
    buf = np.frombuffer(b"".join(parts), np.uint8).copy()
    exp = _oracle_batch(buf, segs, carries)
    L.hvws_set_speculation(eng.ctx, 0)
    _step_checked(eng, buf, segs, carries, *exp, ("exact", 1, 0))          # learns the region size
    for mode in (("slack", 1, 2), ("pipelined_slack", 1, 2)):
        assert _step_checked(eng, buf, segs, carries, *exp, mode) == 5, mode   # HVWS_PATH_SLACK
        f = eng.frames()
        ends = f["pay_off"] + f["pay_len"]
        assert np.all(ends[1:] >= ends[:-1])
    L.hvws_set_speculation(eng.ctx, -1)



