"""GPU: the RUN path of hvws_step / hvws_step_resident (include/hvws.h
hvws_set_run; round 5).  A batch of many segments, each one run of equal
small frames, is unmasked from per-segment run descriptors; the unmask itself
checks every run header against the hypothesis and a repair pass behind it
undoes and redoes exactly any segment that is not one run.  Bytes, frames
(built on demand) and carries must equal the oracle's -- which is the
reference's websocket_parser_execute + decode (http/websocket_parser.c:53-189)
-- for uniform batches, for batches that break the hypothesis anywhere, and
through the automatic adaptation."""
from __future__ import annotations

import random

import numpy as np
import pytest

import libhv_amd
import streams as S
import wsharness as H
from libhv_amd import synth
from test_gpu_parity import _oracle_batch

pytestmark = pytest.mark.gpu

PATH_RUN = 7


def _check(eng, buf, segs, exp_recs, exp_carry, exp_started):
    frames = eng.frames()
    cout, started = eng.carry(len(segs))
    assert len(frames) == len(exp_recs)
    for f in ("hdr_off", "pay_off", "pay_len", "length", "key", "info"):
        assert np.array_equal(frames[f], exp_recs[f]), f
    for s in range(len(segs)):
        assert cout[s].fields() == exp_carry[s].fields(), s
        assert started[s] == exp_started[s], s


@pytest.fixture
def fresh():
    """A context of its own (what earlier tests taught the shared one does not
    leak into the adaptation), with the large-batch path for small batches."""
    e = libhv_amd.Engine(0)
    L = libhv_amd.lib()
    L.hvws_set_fast_bound(e.ctx, 1)
    yield e
    e.close()


def test_run_taken_for_uniform_steps_and_repairs_nothing(fresh):
    """Uniform 1 KiB frames in 24 segments: after the first exact scan sees
    them uniform, steps take RUN; nothing is repaired; every step's bytes,
    frames and carries equal the oracle's."""
    eng, L = fresh, libhv_amd.lib()
    plan = synth.uniform_plan(6000, 1024, 41).split(24)
    host = H.synth_cpu(plan)
    recs, carry, started, exp = _oracle_batch(host, plan.segments, None)
    rx = eng.to_device(host)
    paths = []
    for k in range(5):
        eng.step(rx, plan.total, plan.segments)
        paths.append(L.hvws_last_scan_path(eng.ctx))
        if paths[-1] == PATH_RUN:
            assert L.hvws_last_run_repairs(eng.ctx) == 0
        assert np.array_equal(rx.download(plan.total), exp if k % 2 == 0 else host), k
        _check(eng, host, plan.segments, recs, carry, started)
    rx.free()
    assert paths[0] != PATH_RUN and PATH_RUN in paths[1:3], paths
    assert paths[-1] == PATH_RUN, paths


def test_run_pipelined_same_buffer(fresh):
    """bench.py's loop: hvws_step_resident on one buffer, RUN steps back to
    back (each scan beside the previous unmask), then every byte checked."""
    eng, L = fresh, libhv_amd.lib()
    plan = synth.uniform_plan(20000, 1024, 43).split(64)
    host = H.synth_cpu(plan)
    recs, carry, started, exp = _oracle_batch(host, plan.segments, None)
    dp = libhv_amd.DevicePlan(eng, plan)
    rx = eng.alloc(plan.total + 64)
    eng.synth(rx, plan.total, plan.seed, dp, 0)
    segs = eng.prepare(plan.segments)
    for _ in range(9):
        eng.step_resident(rx, plan.total, segs)
    assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
    eng.sync()
    assert eng.synth(rx, plan.total, plan.seed, dp, 2) == 0   # 9 passes: unmasked
    _check(eng, host, plan.segments, recs, carry, started)
    dp.free()
    rx.free()


@pytest.mark.parametrize("where", ["first", "middle", "last", "tail_then_more"])
def test_run_hypothesis_breaks(fresh, where):
    """One segment that is not one run -- a frame of another size at its
    start, middle or end, or a whole frame after the cut one -- under RUN
    forced: that segment alone is repaired, and bytes, frames and carries
    equal the oracle's."""
    eng, L = fresh, libhv_amd.lib()
    L.hvws_set_run(eng.ctx, 1)
    rng = random.Random(["first", "middle", "last", "tail_then_more"].index(where))
    key = b"\x11\x22\x33\x44"
    segs, parts, at = [], [], 0
    bad = 5
    for s in range(12):
        lens = [1000] * 40
        if s == bad:
            if where == "first":
                lens[1] = 700
            elif where == "middle":
                lens[20] = 1001
            elif where == "last":
                lens[38] = 3   # (a different last frame alone is the cut frame: exact, no failure)
            else:
                lens += [50, 60]
        data = H.build_frames_ref([(0x2 | 0x10 | 0x20, rng.randbytes(n), key) for n in lens])
        parts.append(data)
        segs.append((at, len(data)))
        at += len(data)
    buf = np.frombuffer(b"".join(parts), np.uint8).copy()
    recs, carry, started, exp = _oracle_batch(buf, segs, None)
    rx = eng.to_device(buf)
    eng.step(rx, len(buf), segs)
    assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
    assert L.hvws_last_run_repairs(eng.ctx) == 1
    assert np.array_equal(rx.download(len(buf)), exp)
    _check(eng, buf, segs, recs, carry, started)
    rx.free()


def test_run_auto_falls_back_on_mixed_traffic(fresh):
    """Automatic mode: uniform traffic takes RUN; a mixed batch arriving next
    is still tried as RUN (the last check said uniform), fails, is repaired
    exactly; the steps after it scan exactly (RUN off for a while); all
    results equal the oracle's throughout."""
    eng, L = fresh, libhv_amd.lib()
    up = synth.uniform_plan(5000, 900, 51).split(16)
    uh = H.synth_cpu(up)
    ur, uc, us, ue = _oracle_batch(uh, up.segments, None)
    rx = eng.to_device(uh)
    for k in range(3):
        eng.step(rx, up.total, up.segments)
    assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
    assert np.array_equal(rx.download(up.total), ue)
    rx.free()
    mp = synth.mixed_plan(6 << 20, 52, hi=1 << 17).split(16)
    mh = H.synth_cpu(mp)
    mr, mc, ms, me = _oracle_batch(mh, mp.segments, None)
    rx = eng.to_device(mh)
    eng.step(rx, mp.total, mp.segments)
    assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
    assert L.hvws_last_run_repairs(eng.ctx) > 0
    assert np.array_equal(rx.download(mp.total), me)
    _check(eng, mh, mp.segments, mr, mc, ms)
    eng.step(rx, mp.total, mp.segments)   # the verdict is read: exact again
    assert L.hvws_last_scan_path(eng.ctx) != PATH_RUN
    assert np.array_equal(rx.download(mp.total), mh)
    _check(eng, mh, mp.segments, mr, mc, ms)
    rx.free()


def test_run_carried_and_cut_frames(fresh):
    """Segments that start inside a frame (payload or header carried in) and
    end inside one (payload, header, or a single byte of it), every frame of
    one size between: the carried-in and cut frames are exact in k_head's
    descriptor, the run in between is checked by the unmask."""
    eng, L = fresh, libhv_amd.lib()
    L.hvws_set_run(eng.ctx, 1)
    rng = random.Random(77)
    key = b"\xa1\xb2\xc3\xd4"
    parts, segs, carries, at = [], [], [], 0
    for s in range(30):
        n = rng.choice([126, 1000, 4000])
        data = H.build_frames_ref([(0x2 | 0x10 | 0x20, rng.randbytes(n), key) for _ in range(30)])
        a = rng.randint(0, len(data) // 3)
        b = rng.randint(2 * len(data) // 3, len(data))
        _, st, _, _ = H.scan_segment(data[:a])
        parts.append(data[a:b])
        segs.append((at, b - a))
        carries.append(st)
        at += b - a
    buf = np.frombuffer(b"".join(parts), np.uint8).copy()
    recs, carry, started, exp = _oracle_batch(buf, segs, carries)
    rx = eng.to_device(buf)
    eng.step(rx, len(buf), segs, carries)
    assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
    assert np.array_equal(rx.download(len(buf)), exp)
    _check(eng, buf, segs, recs, carry, started)
    rx.free()


def test_run_random_streams_forced(fresh):
    """Random streams (every opcode, masked and unmasked, all length classes)
    cut into segments, under RUN forced: mostly repaired, always exact."""
    eng, L = fresh, libhv_amd.lib()
    L.hvws_set_run(eng.ctx, 1)
    rng = random.Random(5)
    for trial in range(4):
        parts, segs, at = [], [], 0
        for c in range(rng.randint(2, 30)):
            data = S.rand_stream(rng, rng.randint(1, 25), max_len=rng.choice([30, 400, 5000]))
            parts.append(data)
            segs.append((at, len(data)))
            at += len(data)
        buf = np.frombuffer(b"".join(parts), np.uint8).copy()
        recs, carry, started, exp = _oracle_batch(buf, segs, None)
        rx = eng.to_device(buf)
        eng.step(rx, len(buf), segs)
        assert np.array_equal(rx.download(len(buf)), exp), trial
        _check(eng, buf, segs, recs, carry, started)
        rx.free()


def _segments(parts):
    segs, at = [], 0
    for p in parts:
        segs.append((at, len(p)))
        at += len(p)
    return np.frombuffer(b"".join(parts), np.uint8).copy(), segs


def test_run_small_strides_forced(fresh):
    """Runs of frames of 2-31 bytes (unmasked empty frames: stride 2; masked
    frames of 0-25 payload bytes: 6-31) under RUN forced, several 16 KiB tiles
    each, beside runs of 32-40 B frames.  k_unmask_run's key slots hold the
    frames of strides >= 32 only (a 16 KiB tile of 2-byte frames holds 8192);
    smaller strides are left to the exact repair (run_fast_ok; DESIGN 4.2, the
    round-5 fault analysis).  Bytes, frames and carries equal the oracle's."""
    eng, L = fresh, libhv_amd.lib()
    L.hvws_set_run(eng.ctx, 1)
    rng = random.Random(2031)
    key = b"\x5a\xa5\x3c\xc3"
    parts, small = [], 0
    for stride in [2, 6, 7, 13, 20, 26, 31, 32, 33, 40]:
        if stride == 2:
            frames = [(0x2 | 0x10, b"", None)] * 24000
        else:
            frames = [(0x2 | 0x10 | 0x20, rng.randbytes(stride - 6), key) for _ in range(40000 // stride)]
        parts.append(H.build_frames_ref(frames))
        small += stride < 32
    buf, segs = _segments(parts)
    recs, carry, started, exp = _oracle_batch(buf, segs, None)
    rx = eng.to_device(buf)
    eng.step(rx, len(buf), segs)
    assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
    assert L.hvws_last_run_repairs(eng.ctx) == small   # exact path: every run of stride < 32
    assert np.array_equal(rx.download(len(buf)), exp)
    _check(eng, buf, segs, recs, carry, started)
    rx.free()


def test_run_fewer_segments_after_more(fresh):
    """One context, RUN forced, batches of 30, then 10, then 5 segments into
    the same table set: a batch's words (any / count / workgroups done) sit
    where an earlier, larger batch had segment failure words.  The repair
    zeroes every word it reads, so a later batch sees none of them (a stale
    'done' count published the verdict early; a stale 'any' or count said
    segments failed that did not)."""
    eng, L = fresh, libhv_amd.lib()
    L.hvws_set_run(eng.ctx, 1)
    rng = random.Random(33)
    key = b"\x01\x23\x45\x67"
    for nseg, bad in ((30, {3, 10, 11, 12, 20}), (10, set()), (5, {2}), (10, set())):
        parts = []
        for s in range(nseg):
            lens = [1000] * 40
            if s in bad:
                lens[17] = 555
            parts.append(H.build_frames_ref([(0x2 | 0x10 | 0x20, rng.randbytes(n), key) for n in lens]))
        buf, segs = _segments(parts)
        recs, carry, started, exp = _oracle_batch(buf, segs, None)
        rx = eng.to_device(buf)
        eng.step(rx, len(buf), segs)
        assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
        assert L.hvws_last_run_repairs(eng.ctx) == len(bad), (nseg, bad)
        assert np.array_equal(rx.download(len(buf)), exp), nseg
        _check(eng, buf, segs, recs, carry, started)
        rx.free()


def test_run_repair_key_from_hypothesis_layout(fresh):
    """The round-5 wrong bytes (gpurun_out/pytest_run_r5c.log): a broken run
    whose hypothesised header positions land in payload bytes that parse as a
    longer header (byte 1 = 0xFE: 126-length, masked -> 8 header bytes
    against the run's 6).  Parsed by its own length, that "header"'s key lies
    in bytes the hypothesis XORed, so the repair read another key than the
    unmask had used and the undo left bytes wrong.  Keys are taken at the
    hypothesis' layout (run_key), inside the hypothesised header, which no
    piece of the hypothesis changes."""
    eng, L = fresh, libhv_amd.lib()
    L.hvws_set_run(eng.ctx, 1)

    def frame(n):   # masked binary frame, wire payload bytes all 0xFE
        return bytes([0x82, 0x80 | n]) + b"\x9b\x17\xe2\x4d" + b"\xfe" * n

    parts = []
    for s in range(6):
        lens = [100] * 160   # 17 KB segments: no tile holds a third segment (those go to the repair whole)
        if s % 2:
            lens[5 + 20 * s] = 60   # the frames after it start 40 B before the hypothesis says
        parts.append(b"".join(frame(n) for n in lens))
    buf, segs = _segments(parts)
    recs, carry, started, exp = _oracle_batch(buf, segs, None)
    rx = eng.to_device(buf)
    eng.step(rx, len(buf), segs)
    assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
    assert L.hvws_last_run_repairs(eng.ctx) == 3
    assert np.array_equal(rx.download(len(buf)), exp)
    _check(eng, buf, segs, recs, carry, started)
    rx.free()


def test_unmask_after_run_step(fresh):
    """hvws_unmask after a RUN step XORs every frame again -- by
    the exact table built on demand, not the spent run descriptors (their
    failure words were cleared by the repair, so segments left to the repair
    would have been skipped).  Uniform, broken and small-stride segments."""
    eng, L = fresh, libhv_amd.lib()
    L.hvws_set_run(eng.ctx, 1)
    rng = random.Random(404)
    key = b"\xde\xad\xbe\xef"
    parts = []
    for s in range(8):
        lens = [700] * 30 if s != 3 else [12] * 3000
        if s == 5:
            lens[9] = 333
        parts.append(H.build_frames_ref([(0x2 | 0x10 | 0x20, rng.randbytes(n), key) for n in lens]))
    buf, segs = _segments(parts)
    _, _, _, exp = _oracle_batch(buf, segs, None)
    rx = eng.to_device(buf)
    eng.step(rx, len(buf), segs)
    assert L.hvws_last_scan_path(eng.ctx) == PATH_RUN
    assert np.array_equal(rx.download(len(buf)), exp)
    libhv_amd._check(L.hvws_unmask(eng.ctx, rx.ptr, len(buf)), "hvws_unmask")
    assert np.array_equal(rx.download(len(buf)), buf)   # masked again, every byte
    rx.free()
