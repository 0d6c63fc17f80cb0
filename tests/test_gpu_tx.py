"""GPU, transmit side: hvws_build_frames against
the reference's websocket_build_frame (http/websocket_parser.c:207-256, via
oracle/_ref when built, else the oracle restatement), frame by frame, plus the
size-independent round trip at batch scale: synthesise a masked batch,
unmask it in place with the receive path, rebuild every frame from the
plaintext payloads with the same flags and keys -- the result must be the
original masked batch byte for byte."""
from __future__ import annotations

import numpy as np
import pytest

import libhv_amd
import wsharness as H
from libhv_amd import synth

pytestmark = pytest.mark.gpu

EDGE_LENS = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 125, 126, 127, 128, 4095, 65535, 65536, 65537, 70001]


def _frames(rng, n, lens=None, p_mask=0.6):
    out = []
    for i in range(n):
        ln = int(lens[i]) if lens is not None else int(rng.choice([rng.integers(0, 126), rng.integers(126, 3000),
                                                                   rng.integers(0, 40)]))
        op = int(rng.choice([0, 1, 2, 8, 9, 10, 3, 15]))
        flags = op | (0x10 if rng.random() < 0.8 else 0) | (0x20 if rng.random() < p_mask else 0)
        key = bytes(rng.integers(0, 256, 4, dtype=np.uint8)) if flags & 0x20 else None
        out.append((flags, bytes(rng.integers(0, 256, ln, dtype=np.uint8)), key))
    return out


def _gpu_build(eng, frames, gap_rng=None, with_off=False):
    """Lay payloads out with random gaps (misaligned offsets) and build on the GPU."""
    pay = bytearray()
    offs = []
    for _, p, _k in frames:
        if gap_rng is not None:
            pay += bytes(int(gap_rng.integers(0, 19)))
        offs.append(len(pay))
        pay += p
    flags = [f for f, _, _ in frames]
    mask = [int.from_bytes(k, "little") if k else 0 for _, _, k in frames]
    lens = [len(p) for _, p, _ in frames]
    total = int(synth.frame_size(np.array(flags, dtype=np.uint8), np.array(lens, dtype=np.uint64)).sum()) if frames else 0
    payload = eng.to_device(np.frombuffer(bytes(pay), dtype=np.uint8)) if pay else eng.alloc(16)
    tx = libhv_amd.TxPlan(eng, offs, lens, flags, mask)
    out = eng.alloc(total + 64)
    ooff = eng.alloc(8 * max(len(frames), 1)) if with_off else None
    try:
        n = eng.build_frames(out, total + 64, payload, len(pay), tx, ooff)
        assert n == total
        got = bytes(out.download(n))
        offv = ooff.download(8 * len(frames), np.uint64) if with_off else None
    finally:
        for b in (payload, out, ooff):
            if b is not None:
                b.free()
        tx.free()
    return got, offv


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_build_random_vs_reference(eng, seed):
    rng = np.random.default_rng(seed)
    frames = _frames(rng, 400)
    got, off = _gpu_build(eng, frames, gap_rng=rng, with_off=True)
    assert got == H.build_frames_ref(frames)
    sizes = [len(H.build_frames_ref([f])) for f in frames]
    assert off.tolist() == list(np.cumsum([0] + sizes[:-1]))


@pytest.mark.parametrize("seed", [21, 22])
def test_build_small_frames_vs_reference(eng, seed):
    """Small frames only (every output <= 2026 bytes, 1 KiB-class frames:
    every output tile a boundary tile), misaligned payload offsets, all
    length classes up to the 16-bit one, tiny frames sharing output chunks;
    frame by frame against the reference."""
    rng = np.random.default_rng(seed)
    lens = np.concatenate([rng.integers(0, 20, 300), rng.integers(120, 130, 100), rng.integers(1000, 2019, 300)])
    rng.shuffle(lens)
    frames = _frames(rng, len(lens), lens=lens)
    got, off = _gpu_build(eng, frames, gap_rng=rng, with_off=True)
    assert got == H.build_frames_ref(frames)
    sizes = [len(H.build_frames_ref([f])) for f in frames]
    assert off.tolist() == list(np.cumsum([0] + sizes[:-1]))


def test_build_length_edges(eng):
    rng = np.random.default_rng(7)
    for p_mask in (0.0, 1.0, 0.5):
        frames = _frames(rng, len(EDGE_LENS), lens=EDGE_LENS, p_mask=p_mask)
        got, _ = _gpu_build(eng, frames, gap_rng=rng)
        assert got == H.build_frames_ref(frames)


def test_build_dense_tiny_frames(eng):
    # thousands of frames per 16 KiB output tile: header-only and 1-byte frames
    rng = np.random.default_rng(11)
    frames = _frames(rng, 20000, lens=rng.integers(0, 3, 20000))
    got, _ = _gpu_build(eng, frames)
    assert got == H.build_frames_ref(frames)


def test_build_aligned_large(eng):
    rng = np.random.default_rng(5)
    frames = _frames(rng, 12, lens=[1 << 20] * 4 + [(1 << 20) + 3] * 4 + [200003] * 4, p_mask=0.7)
    got, _ = _gpu_build(eng, frames)
    assert got == H.build_frames_ref(frames)


def test_build_empty_batch(eng):
    tx = libhv_amd.TxPlan(eng, [], [], [], [])
    out = eng.alloc(64)
    try:
        assert eng.build_frames(out, 64, None, 0, tx) == 0
    finally:
        out.free()
        tx.free()


def test_build_rejects_bad_tables(eng):
    pay = eng.alloc(1024)
    out = eng.alloc(4096)
    try:
        tx = libhv_amd.TxPlan(eng, [1000], [100], [0x12], [0])        # payload range past the end
        with pytest.raises(libhv_amd.HvwsError, match="outside"):
            eng.build_frames(out, 4096, pay, 1024, tx)
        tx.free()
        tx = libhv_amd.TxPlan(eng, [0], [10], [0x32])                # masked but no key table
        with pytest.raises(libhv_amd.HvwsError, match="mask"):
            eng.build_frames(out, 4096, pay, 1024, tx)
        tx.free()
        tx = libhv_amd.TxPlan(eng, [0], [1000], [0x12], [0])          # output too small
        with pytest.raises(libhv_amd.HvwsError, match="capacity"):
            eng.build_frames(out, 100, pay, 1024, tx)
        tx.free()
    finally:
        pay.free()
        out.free()


@pytest.mark.parametrize("name,plan", [("mixed", lambda: synth.mixed_plan(1 << 30, 3)),
                                       ("c2", lambda: synth.config_plan("c2", 1))])
def test_build_roundtrip_batch(eng, name, plan):
    """rx unmask then tx build with the same flags/keys == the masked batch."""
    p = plan().split(64)
    dp = libhv_amd.DevicePlan(eng, p)
    rx = eng.alloc(p.total + 64)
    out = eng.alloc(p.total + 64)
    hdr = synth.frame_size(p.flags, p.length) - p.length
    tx = libhv_amd.TxPlan(eng, p.frame_off + hdr, p.length, p.flags, p.mask)
    try:
        eng.synth(rx, p.total, p.seed, dp, 0)
        eng.step(rx, p.total, p.segments)
        assert eng.synth(rx, p.total, p.seed, dp, 2) == 0           # rx holds plaintext payloads
        n = eng.build_frames(out, p.total + 64, rx, p.total, tx)
        assert n == p.total
        assert eng.synth(out, p.total, p.seed, dp, 1) == 0          # rebuilt == masked batch
    finally:
        for b in (rx, out):
            b.free()
        dp.free()
        tx.free()


def _gpu_build_same_offset(eng, frames, rng, move=None):
    """Payloads placed where the output puts them (a relay's layout), the
    bytes between them (the headers' places) random junk the build must not
    copy; `move` = a frame index whose payload is moved one byte instead."""
    L = libhv_amd.lib()
    flags = [f for f, _, _ in frames]
    mask = [int.from_bytes(k, "little") if k else 0 for _, _, k in frames]
    lens = [len(p) for _, p, _ in frames]
    sizes = synth.frame_size(np.array(flags, dtype=np.uint8), np.array(lens, dtype=np.uint64))
    total = int(sizes.sum())
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    hdr = sizes - np.array(lens, dtype=np.uint64)
    offs = (starts + hdr.astype(np.int64)).tolist()
    pay = bytearray(rng.integers(0, 256, total + 32, dtype=np.uint8).tobytes())
    for i, (_, p, _k) in enumerate(frames):
        o = offs[i] + (1 if move == i else 0)
        pay[o:o + len(p)] = p
        offs[i] = o
    payload = eng.to_device(np.frombuffer(bytes(pay), dtype=np.uint8))
    tx = libhv_amd.TxPlan(eng, offs, lens, flags, mask)
    out = eng.alloc(total + 64)
    try:
        n = eng.build_frames(out, total + 64, payload, len(pay), tx)
        assert n == total
        got = bytes(out.download(n))
        kern = L.hvws_last_build_kernel(eng.ctx).decode()
    finally:
        for b in (payload, out):
            b.free()
        tx.free()
    return got, kern


@pytest.mark.parametrize("kind", ["random", "small", "edges", "tiny", "large", "unmasked"])
def test_build_same_offset_layout(eng, kind):
    """Every payload already at its output offset (a relay re-framing what it
    received; round 3 had a kernel of its own for it), frame by frame against
    the reference -- headers written over the junk between payloads, keys at
    every phase, tiles with more frames than LDS holds (tiny) taking the
    chunk-by-chunk fallback."""
    rng = np.random.default_rng(hash(kind) & 0xFFFF)
    if kind == "random":
        frames = _frames(rng, 400)
    elif kind == "small":
        lens = np.concatenate([rng.integers(0, 20, 300), rng.integers(120, 130, 100), rng.integers(1000, 2019, 300)])
        rng.shuffle(lens)
        frames = _frames(rng, len(lens), lens=lens)
    elif kind == "edges":
        frames = _frames(rng, len(EDGE_LENS), lens=EDGE_LENS, p_mask=0.5)
    elif kind == "tiny":
        frames = _frames(rng, 20000, lens=rng.integers(0, 3, 20000))
    elif kind == "large":
        frames = _frames(rng, 12, lens=[1 << 20] * 4 + [(1 << 20) + 3] * 4 + [200003] * 4, p_mask=0.7)
    else:
        frames = _frames(rng, 300, p_mask=0.0)
    got, kern = _gpu_build_same_offset(eng, frames, rng)
    assert got == H.build_frames_ref(frames)
    assert kern.startswith("k_build<"), kern


def test_build_one_moved_payload(eng):
    rng = np.random.default_rng(99)
    frames = _frames(rng, 200, lens=rng.integers(1, 3000, 200))
    got, kern = _gpu_build_same_offset(eng, frames, rng, move=137)
    assert got == H.build_frames_ref(frames)


@pytest.mark.parametrize("v", ["0", "1", "2", "3", "4", "5"])
def test_build_every_geometry(eng, v, monkeypatch):
    """Every k_build geometry ($HVWS_EXPERIMENT build=) builds small frames, edge lengths
    and misaligned payloads byte for byte like the reference and reports its
    name; unset, the pick follows the mean frame size."""
    monkeypatch.setenv("HVWS_EXPERIMENT", f"build={v}")
    L = libhv_amd.lib()
    rng = np.random.default_rng(3)
    lens = np.concatenate([rng.integers(0, 20, 200), rng.integers(1000, 2019, 300), np.array(EDGE_LENS)])
    frames = _frames(rng, len(lens), lens=lens)
    got, _ = _gpu_build(eng, frames, gap_rng=rng)
    assert got == H.build_frames_ref(frames)
    assert L.hvws_last_build_kernel(eng.ctx).decode().startswith("k_build<")


def test_build_geometry_by_frame_size(eng, monkeypatch):
    monkeypatch.delenv("HVWS_EXPERIMENT", raising=False)
    L = libhv_amd.lib()
    rng = np.random.default_rng(4)
    small = _frames(rng, 300, lens=[1000] * 300)
    got, _ = _gpu_build(eng, small)
    assert got == H.build_frames_ref(small)
    assert L.hvws_last_build_kernel(eng.ctx).decode().endswith(",lean>")
    big = _frames(rng, 8, lens=[70001] * 8)
    got, _ = _gpu_build(eng, big)
    assert got == H.build_frames_ref(big)
    assert not L.hvws_last_build_kernel(eng.ctx).decode().endswith(",lean>")


@pytest.mark.parametrize("order", ["packed", "gaps", "shuffled"])
def test_build_boundary_tiles_span_staged(eng, order):
    """Boundary tiles of the general layout stage their source span in LDS
    together with the frame records (k_tx_index).  Small frames packed back
    to back, with gaps, and with payloads in shuffled order (spans past the
    LDS area fall back to the records-first path); every byte against the
    reference."""
    rng = np.random.default_rng(31)
    lens = np.concatenate([rng.integers(900, 1100, 1500), rng.integers(0, 130, 300)])
    rng.shuffle(lens)
    frames = _frames(rng, len(lens), lens=lens, p_mask=0.9)
    if order == "shuffled":
        perm = rng.permutation(len(frames))
        pay = bytearray()
        offs = [0] * len(frames)
        for i in perm:
            offs[i] = len(pay)
            pay += frames[i][1]
        flags = [f for f, _, _ in frames]
        mask = [int.from_bytes(k, "little") if k else 0 for _, _, k in frames]
        lns = [len(p) for _, p, _ in frames]
        total = int(synth.frame_size(np.array(flags, dtype=np.uint8), np.array(lns, dtype=np.uint64)).sum())
        payload = eng.to_device(np.frombuffer(bytes(pay), dtype=np.uint8))
        tx = libhv_amd.TxPlan(eng, offs, lns, flags, mask)
        out = eng.alloc(total + 64)
        try:
            assert eng.build_frames(out, total + 64, payload, len(pay), tx) == total
            got = bytes(out.download(total))
        finally:
            payload.free()
            out.free()
            tx.free()
    else:
        got, _ = _gpu_build(eng, frames, gap_rng=rng if order == "gaps" else None)
    assert got == H.build_frames_ref(frames)


def _build_at(eng, frames, offs, pay: bytes):
    """hvws_build_frames with explicit payload offsets into `pay`; returns the
    output bytes and whether the call took the index-free uniform path."""
    flags = [f for f, _, _ in frames]
    mask = [int.from_bytes(k, "little") if k else 0 for _, _, k in frames]
    lens = [len(p) for _, p, _ in frames]
    total = int(synth.frame_size(np.array(flags, dtype=np.uint8), np.array(lens, dtype=np.uint64)).sum())
    payload = eng.to_device(np.frombuffer(pay, dtype=np.uint8)) if pay else eng.alloc(16)
    tx = libhv_amd.TxPlan(eng, offs, lens, flags, mask)
    out = eng.alloc(total + 64)
    try:
        assert eng.build_frames(out, total + 64, payload, len(pay), tx) == total
        got = bytes(out.download(total))
    finally:
        for b in (payload, out):
            b.free()
        tx.free()
    return got, libhv_amd.lib().hvws_last_build_uniform(eng.ctx)


@pytest.mark.parametrize("ln", [0, 1, 7, 125, 1024, 3000, 70001])
@pytest.mark.parametrize("layout", ["packed", "gap", "rx", "shared", "one"])
def test_build_uniform_layouts(eng, ln, layout):
    """Uniform layouts of small frames (every frame the same size and payload
    length, 256 B to 4 KiB, payload offsets a + k*b with b >= the payload length)
    build without a tile index
    -- each tile finds its frames and source span from its position -- frame by
    frame equal to the reference's websocket_build_frame: payloads packed, with
    a fixed gap, where an rx batch holds them, a single frame; all frames
    sharing one payload (b = 0) take the index and are equal too."""
    rng = np.random.default_rng(ln * 7 + len(layout))
    n = 1 if layout == "one" else max(3, min(3000, (4 << 20) // (ln + 14)))
    fl = 0x2 | 0x10 | 0x20
    body = bytes(rng.integers(0, 256, ln, dtype=np.uint8))
    frames = [(fl, body if layout == "shared" else bytes(rng.integers(0, 256, ln, dtype=np.uint8)),
               bytes(rng.integers(0, 256, 4, dtype=np.uint8))) for _ in range(n)]
    a = int(rng.integers(0, 40))
    step = {"packed": ln, "gap": ln + 13, "rx": len(H.build_frames_ref([frames[0]])),
            "shared": 0, "one": 0}[layout]
    offs = [a + k * step for k in range(n)]
    pay = bytearray(a + (n - 1) * step + ln + 8)
    for k, (_, p, _) in enumerate(frames):
        pay[offs[k]:offs[k] + ln] = p
    got, uni = _build_at(eng, frames, offs, bytes(pay))
    assert got == H.build_frames_ref(frames)
    # one payload shared by every frame (a step shorter than a payload), or
    # frames of 4 KiB and more (the default form, where the index costs ~0.1 %
    # of the call) or under 256 B (the default form too: build_pick): the index
    size = len(H.build_frames_ref([frames[0]]))
    assert uni == (0 if (layout == "shared" and ln) or size >= 4096 or size < 256 else 1)


@pytest.mark.parametrize("kind", ["same_size_other_lengths", "descending", "one_longer", "shuffled"])
def test_build_not_uniform_takes_the_index(eng, kind):
    """Layouts that only look uniform take the tile index and still equal the
    reference: equal sizes from different lengths (masked L, unmasked L + 4),
    descending payload offsets, one frame longer, shuffled offsets."""
    rng = np.random.default_rng(77)
    n, ln = 2000, 1000
    frames = []
    for k in range(n):
        masked = kind != "same_size_other_lengths" or k % 2 == 0
        m = ln + (0 if masked else 4) + (5 if kind == "one_longer" and k == 1234 else 0)
        frames.append((0x2 | 0x10 | (0x20 if masked else 0), bytes(rng.integers(0, 256, m, dtype=np.uint8)),
                       bytes(rng.integers(0, 256, 4, dtype=np.uint8)) if masked else None))
    lens = [len(p) for _, p, _ in frames]
    offs = list(np.concatenate([[0], np.cumsum(lens)[:-1]]))
    if kind in ("descending", "shuffled"):
        perm = list(range(n))[::-1] if kind == "descending" else list(rng.permutation(n))
        pos = np.concatenate([[0], np.cumsum([lens[i] for i in perm])[:-1]])
        offs = [0] * n
        for j, i in enumerate(perm):
            offs[i] = int(pos[j])
        pay = b"".join(frames[i][1] for i in perm)
    else:
        pay = b"".join(p for _, p, _ in frames)
    got, uni = _build_at(eng, frames, [int(o) for o in offs], pay)
    assert got == H.build_frames_ref(frames)
    assert uni == 0
