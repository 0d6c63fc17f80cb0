"""Synthetic masked-frame batch plans.

A plan lists, per frame, where it sits in the rx buffer and what header it
carries (flags, 32-bit key, payload length); the payload bytes themselves
are a pure function of (seed, frame index, byte index) and are written on the
device by hvws_synth (include/hvws_synth.h) or on the CPU by the oracle
(oracle/ws_oracle.c, ows_synth_fill) -- both lay frames out exactly like the
reference's websocket_build_frame (http/websocket_parser.c:207-256).

All randomness here is a splitmix64 stream, so plans are identical on every
machine and numpy version.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

FIN, MASK = 0x10, 0x20
OP_CONT, OP_TEXT, OP_BIN, OP_CLOSE, OP_PING, OP_PONG = 0, 1, 2, 8, 9, 10
GOLD = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def mix64_int(x: int) -> int:
    z = (x + GOLD) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def mix64(x: np.ndarray) -> np.ndarray:
    z = x.astype(np.uint64) + np.uint64(GOLD)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


class SplitMix:
    def __init__(self, seed: int):
        self.s = seed & M64

    def next(self) -> int:
        v = mix64_int(self.s)
        self.s = (self.s + GOLD) & M64
        return v

    def uniform(self) -> float:
        return (self.next() >> 11) / float(1 << 53)

    def randint(self, lo: int, hi: int) -> int:
        """inclusive"""
        return lo + self.next() % (hi - lo + 1)


def frame_size(flags, length):
    """websocket_calc_frame_size (reference http/websocket_parser.c:191-205), vectorised."""
    length = np.asarray(length, dtype=np.uint64)
    flags = np.asarray(flags)
    ext = np.where(length < 126, 0, np.where(length <= 0xFFFF, 2, 8)).astype(np.uint64)
    m = np.where((flags & MASK) != 0, 4, 0).astype(np.uint64)
    return length + np.uint64(2) + ext + m


def frame_keys(seed: int, n: int) -> np.ndarray:
    i = np.arange(n, dtype=np.uint64)
    return (mix64(i ^ np.uint64(seed * 0x5851F42D4C957F2D & M64)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


@dataclass
class Plan:
    seed: int
    frame_off: np.ndarray
    flags: np.ndarray
    mask: np.ndarray
    length: np.ndarray
    text: Optional[np.ndarray]
    total: int
    segments: List[Tuple[int, int]] = field(default_factory=list)

    @property
    def n(self) -> int:
        return int(self.length.shape[0])

    @property
    def payload_bytes(self) -> int:
        return int(self.length.sum())

    @property
    def header_bytes(self) -> int:
        return int((frame_size(self.flags, self.length) - self.length).sum())

    def masked_payload_bytes(self) -> int:
        return int(self.length[(self.flags & MASK) != 0].sum())

    def split(self, nseg: int) -> "Plan":
        """Cut the back-to-back frames into nseg segments (connections) at frame
        boundaries, ~equal frame counts each."""
        nseg = max(1, min(nseg, self.n)) if self.n else 1
        sizes = frame_size(self.flags, self.length)
        bounds = np.linspace(0, self.n, nseg + 1).astype(np.int64)
        segs = []
        for s in range(nseg):
            a, b = int(bounds[s]), int(bounds[s + 1])
            if a >= b:
                continue
            off = int(self.frame_off[a])
            end = int(self.frame_off[b - 1] + sizes[b - 1])
            segs.append((off, end - off))
        self.segments = segs or [(0, self.total)]
        return self


def uniform_plan(n: int, payload: int, seed: int, opcode: int = OP_BIN, text: bool = False,
                 masked: bool = True) -> Plan:
    """n frames of `payload` bytes, FIN set, back to back from offset 0."""
    fl = opcode | FIN | (MASK if masked else 0)
    flags = np.full(n, fl, dtype=np.uint8)
    length = np.full(n, payload, dtype=np.uint64)
    size = int(frame_size(np.array([fl]), np.array([payload], dtype=np.uint64))[0])
    frame_off = np.arange(n, dtype=np.uint64) * np.uint64(size)
    mask = frame_keys(seed, n)
    tx = np.full(n, 1 if text else 0, dtype=np.uint8)
    p = Plan(seed, frame_off, flags, mask, length, tx, n * size)
    p.segments = [(0, n * size)]
    return p


def mixed_plan(target_bytes: int, seed: int, lo: int = 128, hi: int = 1 << 20, frag_prob: float = 0.25,
               ping_prob: float = 0.03) -> Plan:
    """Config 4: log-uniform payloads in [lo, hi], ~frag_prob of messages split in
    2-8 fragments (FIN=0 then CONTINUE frames), PING control frames (<=125 B,
    6-byte headers) between messages."""
    r = SplitMix(seed ^ 0xC0FFEE)
    flags: List[int] = []
    length: List[int] = []
    text: List[int] = []
    total = 0
    import math

    span = math.log2(hi) - math.log2(lo)
    while total < target_bytes:
        if r.uniform() < ping_prob:
            L = r.randint(0, 125)
            flags.append(OP_PING | FIN | MASK)
            length.append(L)
            text.append(0)
            total += L + 6
            continue
        L = int(2 ** (math.log2(lo) + span * r.uniform()))
        L = max(lo, min(hi, L))
        op = OP_TEXT if r.uniform() < 0.5 else OP_BIN
        tx = 1 if op == OP_TEXT else 0
        if r.uniform() < frag_prob and L >= 8:
            k = r.randint(2, 8)
            cuts = sorted(set(r.randint(1, L - 1) for _ in range(k - 1)))
            parts = [b - a for a, b in zip([0] + cuts, cuts + [L])]
        else:
            parts = [L]
        for i, pl in enumerate(parts):
            f = (op if i == 0 else OP_CONT) | MASK
            if i == len(parts) - 1:
                f |= FIN
            flags.append(f)
            length.append(pl)
            text.append(tx)
            total += int(frame_size(np.array([f]), np.array([pl], dtype=np.uint64))[0])
    fl = np.array(flags, dtype=np.uint8)
    ln = np.array(length, dtype=np.uint64)
    sizes = frame_size(fl, ln)
    off = np.zeros(len(ln), dtype=np.uint64)
    if len(ln):
        off[1:] = np.cumsum(sizes)[:-1]
    p = Plan(seed, off, fl, frame_keys(seed, len(ln)), ln, np.array(text, dtype=np.uint8), int(sizes.sum()))
    p.segments = [(0, p.total)]
    return p


def config_plan(name: str, seed: int = 1) -> Plan:
    """BASELINE.json configs (full size)."""
    if name == "c1":
        return uniform_plan(1000, 1024, seed, opcode=OP_TEXT, text=True)
    if name == "c2":
        return uniform_plan(1 << 20, 1024, seed)
    if name == "c3":
        return uniform_plan(1 << 20, 65536, seed)
    if name == "c4":
        return mixed_plan(4 << 30, seed)
    raise KeyError(name)
