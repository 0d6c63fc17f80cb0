"""GPU: lagged steps (include/hvws.h hvws_lagged_*; round 5): consecutive
hvws_step_resident steps on two contexts from two worker threads, so two scan
chains are in flight; unmasks stay in call order.  Bytes after hvws_lagged_sync
must equal the oracle's -- the reference's websocket_parser_execute + decode
(http/websocket_parser.c:53-189) -- for one long mixed stream (the frame
sieve's path, config 4 as one stream), for many connections, for one buffer
stepped over and over (two unmasks of it racing would corrupt it), and at full
config-4 size against the reference digest."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import libhv_amd
import wsharness as H
from libhv_amd import synth
from test_gpu_parity import _oracle_batch

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs.json")))


@pytest.fixture
def lag(eng):
    libhv_amd.lib().hvws_set_sieve_min(0)   # the default threshold (8 MiB)
    with eng.lagged() as g:
        yield g


@pytest.mark.parametrize("steps", [1, 2, 5, 8])
def test_lagged_one_buffer_in_order(eng, lag, steps):
    """One 24 MiB stream of mixed 128 B-256 KiB frames (one segment: the frame
    sieve), stepped `steps` times through the lagged stepper: an odd count
    leaves it unmasked, an even one masked, byte for byte."""
    plan = synth.mixed_plan(24 << 20, 61, hi=1 << 18).split(1)
    host = H.synth_cpu(plan)
    _, _, _, exp = _oracle_batch(host, plan.segments, None)
    rx = eng.to_device(host)
    segs = eng.prepare(plan.segments)
    for _ in range(steps):
        lag.step(rx, plan.total, segs)
    lag.sync()
    assert np.array_equal(rx.download(plan.total), exp if steps % 2 else host)
    rx.free()


def test_lagged_distinct_buffers(eng, lag):
    """Three batches of different shapes (one mixed stream, 37 mixed
    connections, 64 connections of uniform 1 KiB frames), stepped A B C A B:
    A masked again, B masked again, C unmasked."""
    plans = [synth.mixed_plan(12 << 20, 71, hi=1 << 17).split(1),
             synth.mixed_plan(8 << 20, 72, hi=1 << 16).split(37),
             synth.uniform_plan(8000, 1024, 73).split(64)]
    hosts = [H.synth_cpu(p) for p in plans]
    exps = [_oracle_batch(h, p.segments, None)[3] for h, p in zip(hosts, plans)]
    rxs = [eng.to_device(h) for h in hosts]
    segs = [eng.prepare(p.segments) for p in plans]
    for k in [0, 1, 2, 0, 1]:
        lag.step(rxs[k], plans[k].total, segs[k])
    lag.sync()
    assert np.array_equal(rxs[0].download(plans[0].total), hosts[0])
    assert np.array_equal(rxs[1].download(plans[1].total), hosts[1])
    assert np.array_equal(rxs[2].download(plans[2].total), exps[2])
    for r in rxs:
        r.free()


def test_lagged_carries_in(eng, lag):
    """Segments that start inside a frame: the carry tables are copied at the
    call, so the caller may reuse them at once."""
    plan = synth.mixed_plan(6 << 20, 81, hi=1 << 16).split(20)
    host = H.synth_cpu(plan)
    # cut every segment's first 100 bytes off: they become each segment's carry
    segs, carries, parts, at = [], [], [], 0
    for o, n in plan.segments:
        _, st, _, _ = H.scan_segment(host[o:o + min(100, n)].tobytes())
        parts.append(host[o + min(100, n):o + n])
        segs.append((at, n - min(100, n)))
        carries.append(st)
        at += n - min(100, n)
    buf = np.concatenate(parts)
    _, _, _, exp = _oracle_batch(buf, segs, carries)
    rx = eng.to_device(buf)
    for _ in range(3):
        lag.step(rx, len(buf), segs, carries)
    lag.sync()
    assert np.array_equal(rx.download(len(buf)), exp)
    rx.free()


def test_lagged_error_sticks(eng, lag):
    """A step the library refuses (an rx pointer not 16-byte aligned) fails
    the stepper: that call or a later one, and sync, report it."""
    plan = synth.uniform_plan(100, 1024, 91).split(1)
    host = H.synth_cpu(plan)
    rx = eng.to_device(np.concatenate([np.zeros(16, np.uint8), host]))

    class Off:
        ptr = rx.ptr + 3

    with pytest.raises(libhv_amd.HvwsError):
        lag.step(Off, plan.total, plan.segments)
        lag.sync()
    with pytest.raises(libhv_amd.HvwsError):
        lag.sync()
    rx.free()


def test_lagged_config4_one_stream_full_size(eng, lag):
    """Config 4 (4.3 GB of mixed 128 B-1 MiB frames) as one stream, 3 lagged
    steps: unmasked, and its digest is the reference's."""
    plan = synth.config_plan("c4", seed=1).split(1)
    dp = libhv_amd.DevicePlan(eng, plan)
    rx = eng.alloc(plan.total + 64)
    try:
        eng.synth(rx, plan.total, plan.seed, dp, 0)
        assert f"{eng.digest(rx, plan.total):016x}" == GOLD["c4"]["digest_masked"]
        segs = eng.prepare(plan.segments)
        for _ in range(3):
            lag.step(rx, plan.total, segs)
        lag.sync()
        assert eng.synth(rx, plan.total, plan.seed, dp, 2) == 0
        assert f"{eng.digest(rx, plan.total):016x}" == GOLD["c4"]["digest_unmasked"]
    finally:
        dp.free()
        rx.free()
