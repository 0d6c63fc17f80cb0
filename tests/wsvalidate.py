"""Test infrastructure: the RFC 6455 validation oracle for hvws_set_validation
(SURVEY.md sec. 8(f) row 4).  The reference validates nothing (SURVEY
Q1-Q4), so these rules come from the RFC, not from libhv:

  V_RSV      sec. 5.2  RSV1-3 MUST be 0 unless an extension is negotiated
  V_OPCODE   sec. 5.2  opcodes 3-7 and 0xB-0xF are reserved
  V_CONTROL  sec. 5.5  control frames MUST have payload <= 125 and MUST NOT be fragmented
  V_LEN64    sec. 5.2  the most significant bit of a 64-bit length MUST be 0
  V_NONMIN   sec. 5.2  the minimal number of bytes MUST be used to encode the length
  V_UNMASKED sec. 5.1  a server MUST close on a frame from the client that is not masked

`make_frame` builds frames that may break any of them; `violations` walks a
byte stream of whole frames and returns each header's offset and classes.
"""
from __future__ import annotations

import random
import struct
from typing import List, Tuple

V_RSV, V_OPCODE, V_CONTROL, V_LEN64, V_NONMIN, V_UNMASKED = 1, 2, 4, 8, 16, 32
V_ALL = 63


def make_frame(rng: random.Random, p_bad: float = 0.3, max_len: int = 3000) -> Tuple[bytes, int]:
    """One frame (bytes) and the classes it violates."""
    bad = rng.random() < p_bad
    viol = 0
    op = rng.choice([0, 1, 2, 8, 9, 10])
    fin = 1
    rsv = 0
    masked = True
    n = rng.randrange(0, 126) if op & 8 else rng.choice([rng.randrange(0, 126), rng.randrange(126, max_len)])
    enc = 0 if n < 126 else (1 if n <= 0xFFFF else 2)
    if bad:
        kind = rng.choice(["rsv", "op", "ctl_fin", "ctl_len", "nonmin", "unmasked", "two"])
        if kind in ("rsv", "two"):
            rsv = rng.randrange(1, 8)
        if kind in ("op", "two"):
            op = rng.choice([3, 4, 5, 6, 7, 11, 12, 13, 14, 15])
        if kind == "ctl_fin":
            op = rng.choice([8, 9, 10])
            fin = 0
        if kind == "ctl_len":
            op = rng.choice([8, 9, 10])
            n = rng.randrange(126, 400)
            enc = 1
        if kind == "nonmin":
            n = rng.randrange(0, 126) if rng.random() < 0.5 else rng.randrange(126, 2000)
            enc = 1 if n < 126 else 2
        if kind == "unmasked":
            masked = False
    if not (op & 8):
        fin = rng.randrange(2) if not bad else fin
    if rsv:
        viol |= V_RSV
    if op in (3, 4, 5, 6, 7) or op >= 11:
        viol |= V_OPCODE
    if (op & 8) and (not fin or n > 125):
        viol |= V_CONTROL
    if (enc == 1 and n < 126) or (enc == 2 and n <= 0xFFFF):
        viol |= V_NONMIN
    if not masked:
        viol |= V_UNMASKED
    b0 = (fin << 7) | (rsv << 4) | op
    len7 = n if enc == 0 else (126 if enc == 1 else 127)
    hdr = bytes([b0, (0x80 if masked else 0) | len7])
    if enc == 1:
        hdr += struct.pack(">H", n)
    elif enc == 2:
        hdr += struct.pack(">Q", n)
    if masked:
        hdr += rng.randbytes(4)
    return hdr + rng.randbytes(n), viol


def len64_msb_frame() -> Tuple[bytes, int]:
    """A header announcing 2^63 + 3 bytes (the parser then waits in its body
    state forever): put it last in a stream."""
    return bytes([0x82, 0xFF]) + struct.pack(">Q", (1 << 63) + 3) + b"\x01\x02\x03\x04", V_LEN64


def violations(data: bytes) -> List[Tuple[int, int]]:
    """(header offset, classes) of every frame whose header is whole in data."""
    out = []
    i = 0
    while i + 2 <= len(data):
        b0, b1 = data[i], data[i + 1]
        op, fin, rsv = b0 & 15, b0 >> 7, (b0 >> 4) & 7
        masked, len7 = b1 >> 7, b1 & 127
        h = 2
        if len7 == 126:
            if i + 4 > len(data):
                break
            n = struct.unpack_from(">H", data, i + 2)[0]
            h += 2
        elif len7 == 127:
            if i + 10 > len(data):
                break
            n = struct.unpack_from(">Q", data, i + 2)[0]
            h += 8
        else:
            n = len7
        h += 4 if masked else 0
        if i + h > len(data):
            break
        v = 0
        v |= V_RSV if rsv else 0
        v |= V_OPCODE if (op in (3, 4, 5, 6, 7) or op >= 11) else 0
        v |= V_CONTROL if (op & 8) and (not fin or n > 125) else 0
        v |= V_LEN64 if (len7 == 127 and n >> 63) else 0
        v |= V_NONMIN if ((len7 == 126 and n < 126) or (len7 == 127 and n <= 0xFFFF)) else 0
        v |= V_UNMASKED if not masked else 0
        out.append((i, v))
        i += h + n
    return out


def random_stream(seed: int, nframes: int, p_bad: float = 0.3, tail_len64: bool = False) -> Tuple[bytes, list]:
    rng = random.Random(seed)
    parts, viol = [], []
    for _ in range(nframes):
        b, v = make_frame(rng, p_bad)
        parts.append(b)
        viol.append(v)
    if tail_len64:
        b, v = len64_msb_frame()
        parts.append(b)
        viol.append(v)
    return b"".join(parts), viol
