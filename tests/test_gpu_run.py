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


@pytest.fixture(params=range(6), ids=lambda g: f"geom{g}")
def geom(request):
    """Every compiled RUN unmask geometry (hvws_set_run_geometry), the default
    (0: 256 x 4, tile staged in LDS) first."""
    L = libhv_amd.lib()
    if request.param >= L.hvws_run_geometry_count():
        pytest.skip("geometry not compiled")
    old = L.hvws_set_run_geometry(request.param)
    yield request.param
    L.hvws_set_run_geometry(old)


@pytest.fixture
def fresh():
    """A context of its own (what earlier tests taught the shared one does not
    leak into the adaptation), with the large-batch path for small batches."""
    e = libhv_amd.Engine(0)
    L = libhv_amd.lib()
    L.hvws_set_fast_bound(e.ctx, 1)
    yield e
    e.close()


def test_run_taken_for_uniform_steps_and_repairs_nothing(geom, fresh):
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
def test_run_hypothesis_breaks(geom, fresh, where):
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


def test_run_carried_and_cut_frames(geom, fresh):
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


def test_run_random_streams_forced(geom, fresh):
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
