"""Seeded WebSocket byte streams for parity tests (all built with the
reference's websocket_build_frame layout; see wsharness.build_frames_ref)."""
from __future__ import annotations

import random
from typing import List, Optional, Sequence, Tuple

import wsharness as H

FIN, MASK = 0x10, 0x20

# payload lengths straddling every header-size boundary
EDGE_LENS = [0, 1, 2, 3, 4, 5, 7, 124, 125, 126, 127, 128, 255, 256, 65534, 65535, 65536, 65537]


def rand_frames(rng: random.Random, nf: int, max_len: int = 300, edge: bool = True,
                unmasked_prob: float = 0.15) -> List[Tuple[int, bytes, Optional[bytes]]]:
    out = []
    for _ in range(nf):
        if edge and rng.random() < 0.3:
            L = rng.choice([x for x in EDGE_LENS if x <= max(max_len, 0)] or [0])
        else:
            L = rng.randint(0, max_len)
        op = rng.choice([0, 1, 2, 8, 9, 10, 3, 0xB, 0xF])
        fl = op | (FIN if rng.random() < 0.75 else 0) | (0 if rng.random() < unmasked_prob else MASK)
        key = bytes(rng.randrange(256) for _ in range(4))
        out.append((fl, rng.randbytes(L), key))
    return out


def rand_stream(rng: random.Random, nf: int, max_len: int = 300, **kw) -> bytes:
    return H.build_frames_ref(rand_frames(rng, nf, max_len, **kw))


def rand_chunks(rng: random.Random, n: int, mode: Optional[str] = None) -> List[int]:
    mode = mode or rng.choice(["one", "rand", "small", "bytes"])
    if mode == "one":
        return [max(n, 1)]
    out, tot = [], 0
    while tot < n:
        c = 1 if mode == "bytes" else (rng.randint(1, 13) if mode == "small" else rng.randint(1, 9000))
        out.append(c)
        tot += c
    return out


def with_rsv(data: bytes, at: int = 0) -> bytes:
    """Set RSV1-3 on the frame header at `at` (Q1: silently dropped)."""
    b = bytearray(data)
    b[at] |= 0x70
    return bytes(b)


def quirk_streams() -> List[Tuple[str, bytes]]:
    """Streams for the reference quirks of SURVEY.md Appendix A."""
    k = bytes([0x37, 0xFA, 0x21, 0x3D])
    B = H.build_frames_ref
    out = [
        ("rfc_hello_masked", bytes.fromhex("818537fa213d7f9f4d5158")),
        ("rfc_hello_unmasked", bytes.fromhex("810548656c6c6f")),
        ("q1_rsv_bits", with_rsv(B([(1 | FIN | MASK, b"rsv", k)]))),
        ("q2_reserved_opcodes", B([(3 | FIN | MASK, b"three", k), (0xB | FIN | MASK, b"eleven", k)])),
        ("q3_unmasked_client", B([(2 | FIN, b"raw bytes", None)])),
        ("q4_nonminimal_126", bytes([0x82, 0xFE, 0x00, 0x03]) + k + bytes(a ^ b for a, b in zip(b"abc", k))),
        ("q4_nonminimal_127", bytes([0x82, 0xFF, 0, 0, 0, 0, 0, 0, 0, 2]) + k + bytes(a ^ b for a, b in zip(b"xy", k))),
        ("q4_len_2p63", bytes([0x82, 0xFF, 0x80, 0, 0, 0, 0, 0, 0, 3]) + k + b"abcdefgh"),
        ("q4_big_control", B([(9 | FIN | MASK, b"p" * 300, k)])),
        ("q4_nonfin_control", B([(9 | MASK, b"ping", k), (0 | FIN | MASK, b"!", k)])),
        ("q5_control_between_fragments",
         B([(1 | MASK, b"AB", k), (9 | FIN | MASK, b"PING", k), (0 | FIN | MASK, b"CD", k)])),
        ("q6_lone_continue", B([(0 | FIN | MASK, b"orphan", k)])),
        ("q7_zero_length", B([(1 | FIN | MASK, b"", k), (2 | FIN, b"", None), (2 | FIN | MASK, b"x", k)])),
        ("q10_inplace", bytes.fromhex("818511223344") + bytes(a ^ b for a, b in zip(b"Hello", bytes.fromhex("1122334411")))),
        ("q14_unmasked_after_masked", B([(1 | FIN | MASK, b"one", k), (2 | FIN, b"two", None), (1 | FIN, b"", None)])),
        ("fragments", B([(1 | MASK, b"He", k), (0 | MASK, b"ll", k), (0 | FIN | MASK, b"o!", k)])),
        ("zero_key", B([(2 | FIN | MASK, b"\x00" * 40, b"\x00\x00\x00\x00")])),
        ("hdr_64k_boundary", B([(2 | FIN | MASK, bytes(65535), k), (2 | FIN | MASK, bytes(65536), k)])),
        ("empty", b""),
    ]
    return out
