"""GPU, BASELINE.json configurations at full size.  The oracle cannot replay
68 GB in seconds, so full-size checks use size-independent properties plus
the reference digests in tests/golden/configs.json:
  * device generator == reference-built batch (digest of the masked bytes);
  * after one pass every payload byte equals its plaintext and every header
    byte is untouched (hvws_synth VERIFY_PLAIN, a byte-exact check);
  * a second pass restores the masked batch exactly (XOR involution);
  * the masked and unmasked digests equal the reference's (configs 1-4, and
    the eight config-5 rank batches bench.py builds: tests/golden/configs.json,
    c3 and c5_rank* streamed through the reference by make_golden.py --big);
  * one frame record per frame."""
from __future__ import annotations

import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import libhv_amd
import wsharness as H
from libhv_amd import synth

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs.json")))


_RX = {}


def _rx(eng, nbytes):
    """One device buffer per size, reused by every test of this module: the
    driver clears freed VRAM in the background, so freeing and reallocating a
    68.7 GB batch per test ran out of memory by the third c3-sized test."""
    b = _RX.get(nbytes)
    if b is None or b.eng is not eng:
        b = _RX[nbytes] = eng.alloc(nbytes)
    return b


@pytest.fixture(scope="module", autouse=True)
def _free_buffers():
    yield
    for b in _RX.values():
        b.free()
    _RX.clear()


def _run(eng, plan, nseg, golden=None, sieve=None, path2=None):
    """sieve: assert the frame sieve's chain covered every frame (one segment);
    path2: the HVWS_PATH_* the second step must take."""
    L = libhv_amd.lib()
    if sieve:
        L.hvws_set_sieve_min(0)   # default threshold; contexts forget "uniform, skip the sieve"
    plan.split(nseg)
    dp = libhv_amd.DevicePlan(eng, plan)
    rx = _rx(eng, plan.total + 64)
    try:
        eng.synth(rx, plan.total, plan.seed, dp, 0)
        if golden:
            assert f"{eng.digest(rx, plan.total):016x}" == golden["digest_masked"]
        eng.step(rx, plan.total, plan.segments)
        assert eng.synth(rx, plan.total, plan.seed, dp, 2) == 0      # plaintext + untouched headers
        if sieve:
            out = (ctypes.c_uint64 * 4)()
            assert L.hvws_last_sieve(eng.ctx, out) == 0
            assert out[0] == 1 and out[2] == plan.n and out[3] == plan.total, list(out)
        assert libhv_amd.lib().hvws_frame_count(eng.ctx) == plan.n
        first, cnt = eng.segment_frames(len(plan.segments))
        assert int(cnt.sum()) == plan.n
        if golden:
            assert f"{eng.digest(rx, plan.total):016x}" == golden["digest_unmasked"]
        carry, _ = eng.carry(len(plan.segments))
        assert all(c.state == 0 and c.require == 0 for c in carry)
        eng.step(rx, plan.total, plan.segments)
        assert eng.synth(rx, plan.total, plan.seed, dp, 1) == 0      # masked again, byte-exact
        if path2 is not None:
            assert L.hvws_last_scan_path(eng.ctx) == path2
    finally:
        dp.free()


@pytest.mark.parametrize("nseg", [1, 4096])
def test_config2_1m_x_1k(eng, nseg):
    _run(eng, synth.config_plan("c2", seed=1), nseg, GOLD["c2"])


@pytest.mark.parametrize("pipelined", [False, True])
def test_config2_run_full_size(eng, pipelined):
    """Config 2 at full size (1M x 1 KiB, 4096 connections) on the RUN path
    (every header read once, inside the unmask), as bench.py
    --config c2 measures it: steps until the RUN path is taken (it needs a
    matched check first), then the reference's unmasked digest after that
    step and its masked digest after the next RUN step, nothing repaired,
    and the on-demand frame records of a RUN step (hvws_frame_count) exact."""
    L = libhv_amd.lib()
    plan = synth.config_plan("c2", seed=1)
    plan.split(4096)
    dp = libhv_amd.DevicePlan(eng, plan)
    rx = _rx(eng, plan.total + 64)
    segs = eng.prepare(plan.segments)
    step = eng.step_resident if pipelined else eng.step
    try:
        eng.synth(rx, plan.total, plan.seed, dp, 0)
        passes = 0
        for _ in range(8):
            step(rx, plan.total, segs)
            passes += 1
            if L.hvws_last_scan_path(eng.ctx) == 7:   # HVWS_PATH_RUN
                break
        assert L.hvws_last_scan_path(eng.ctx) == 7, "RUN was not taken on a uniform c2 batch"
        eng.sync()
        assert L.hvws_last_run_repairs(eng.ctx) == 0
        want = GOLD["c2"]["digest_unmasked" if passes % 2 else "digest_masked"]
        assert f"{eng.digest(rx, plan.total):016x}" == want
        step(rx, plan.total, segs)
        passes += 1
        assert L.hvws_last_scan_path(eng.ctx) == 7
        eng.sync()
        want = GOLD["c2"]["digest_unmasked" if passes % 2 else "digest_masked"]
        assert f"{eng.digest(rx, plan.total):016x}" == want
        assert eng.synth(rx, plan.total, plan.seed, dp, 2 if passes % 2 else 1) == 0
        assert L.hvws_frame_count(eng.ctx) == plan.n   # records built on demand (run_materialize)
    finally:
        dp.free()


@pytest.mark.parametrize("nseg", [4096, 1])
def test_config3_1m_x_64k(eng, nseg):
    _run(eng, synth.config_plan("c3", seed=1), nseg, GOLD["c3"])


@pytest.mark.parametrize("rank", range(8))
def test_config5_rank_batches(eng, rank):
    """Config 5 (8M x 64 KiB over 8 GPUs) is eight disjoint c3-shaped batches,
    one per rank (bench.py rank_plan: seed 1000 + rank).  Each one, on this
    GPU, against its reference digests."""
    _run(eng, synth.config_plan("c3", seed=1000 + rank), 4096, GOLD[f"c5_rank{rank}"])


@pytest.mark.parametrize("nseg", [1, 1024, 4096])
def test_config4_mixed(eng, nseg):
    """One stream: the frame sieve discovers all 74 701 frames; 1024 and 4096
    connections (4096: bench.py's default): the second step takes the SLACK
    table, whose walk then runs several segments per wave (the grid cap of a
    SLACK scan, hvws_engine.cpp)."""
    _run(eng, synth.config_plan("c4", seed=1), nseg, GOLD["c4"], sieve=nseg == 1,
         path2=5 if nseg > 1 else None)


def test_config1_through_websocketparser_8k_chunks():
    """Config 1 end to end through the drop-in WebSocketParser::FeedRecvData,
    fed in 8 KiB event-loop chunks (event/hevent.h:16)."""
    g = GOLD["c1"]
    plan = synth.config_plan("c1", seed=1)
    data = H.synth_cpu(plan).tobytes()
    assert hashlib.sha256(data).hexdigest() == g["sha256_masked"]
    msgs, rets, state, buf = H.run_messages("gpu", data, [8192] * ((len(data) + 8191) // 8192))
    assert len(msgs) == g["messages"] == 1000
    assert sum(len(m) for _, m in msgs) == g["message_bytes"]
    assert sum(op * 31 + (m[-1] if m else 0) for op, m in msgs) == g["message_xsum"]
    assert all(op == 1 for op, _ in msgs)
    assert hashlib.sha256(buf).hexdigest() == g["sha256_unmasked"]
    assert rets == [8192] * (len(data) // 8192) + ([len(data) % 8192] if len(data) % 8192 else [])
