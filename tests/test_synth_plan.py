"""CPU: synthetic batch plans (host logic behind bench.py and the GPU tests)."""
from __future__ import annotations

import numpy as np

import wsharness as H
from libhv_amd import synth


def test_frame_size_matches_reference_rule():
    O = H.oracle()
    for n in [0, 1, 125, 126, 127, 65535, 65536, 1 << 20, (1 << 32) + 5]:
        for fl in (0x22, 0x02, 0x39):
            assert int(synth.frame_size(np.array([fl]), np.array([n], np.uint64))[0]) == O.ows_calc_frame_size(fl, n)


def test_uniform_plan_layout():
    p = synth.config_plan("c3")
    assert p.n == 1 << 20
    assert p.total == (1 << 20) * 65550
    assert p.payload_bytes == 1 << 36
    assert p.header_bytes == 14 << 20
    p2 = synth.config_plan("c2")
    assert p2.total == 1_082_130_432 and p2.header_bytes == 8 << 20
    p1 = synth.config_plan("c1")
    assert p1.total == 1_032_000 and set(p1.flags.tolist()) == {0x31}


def test_split_segments_cover_frames():
    p = synth.mixed_plan(32 << 20, 3).split(37)
    sizes = synth.frame_size(p.flags, p.length)
    assert sum(n for _, n in p.segments) == p.total
    starts = set(int(x) for x in p.frame_off)
    for off, n in p.segments:
        assert off in starts
    assert all(a[0] + a[1] == b[0] for a, b in zip(p.segments, p.segments[1:]))
    assert int(sizes.sum()) == p.total


def test_mixed_plan_properties():
    """Config 4 shape: all three header sizes, FIN=0 fragments closed by a FIN
    CONTINUE, PING control frames between messages, payloads in [128, 1 MiB]."""
    p = synth.mixed_plan(64 << 20, 9)
    hl = synth.frame_size(p.flags, p.length) - p.length
    assert {6, 8, 14} <= set(int(x) for x in np.unique(hl))
    op = p.flags & 0x0F
    fin = (p.flags & 0x10) != 0
    assert (op == 0).any() and (~fin).any() and (op == 9).any()
    data = p.length[op != 9]
    assert data.max() <= 1 << 20
    # every non-FIN run ends with a FIN CONTINUE frame
    open_msg = False
    for o, f in zip(op.tolist(), fin.tolist()):
        if o == 9:
            continue
        if open_msg:
            assert o == 0
        else:
            assert o in (1, 2)
        open_msg = not f
    assert not open_msg


def test_plans_deterministic_and_rank_distinct():
    a = synth.mixed_plan(8 << 20, 5)
    b = synth.mixed_plan(8 << 20, 5)
    assert np.array_equal(a.length, b.length) and np.array_equal(a.mask, b.mask)
    r0 = synth.config_plan("c2", seed=1000)
    r1 = synth.config_plan("c2", seed=1001)
    assert not np.array_equal(r0.mask, r1.mask)


def test_oracle_synth_matches_reference_build(tmp_path):
    if not H.have_ref():
        import pytest

        pytest.skip("reference library not built here")
    plan = synth.mixed_plan(2 << 20, 12, hi=1 << 17)
    buf = H.synth_cpu(plan)
    frames = []
    O = H.oracle()
    import ctypes

    for i in range(plan.n):
        n = int(plan.length[i])
        t = ctypes.create_string_buffer(max(n, 1))
        O.ows_synth_plain(t, plan.seed, i, n, int(plan.text[i]))
        frames.append((int(plan.flags[i]), t.raw[:n], int(plan.mask[i]).to_bytes(4, "little")))
    assert H.build_frames_ref(frames) == buf.tobytes()
