"""GPU, batched handshake digest (hvws_encode_keys) against the reference
ws_encode_key fixture (tests/golden/ws_keys.json), the RFC 6455 sec. 1.3 known
answer, and -- at batch scale -- the library's host ws_encode_key on random
keys of every length class."""
from __future__ import annotations

import base64
import ctypes
import json
import os
import random

import pytest

import libhv_amd

pytestmark = pytest.mark.gpu
CASES = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ws_keys.json")))["cases"]


def test_keys_match_reference_fixture(eng):
    got = eng.encode_keys([k.encode() for k, _ in CASES])
    for (k, a), g in zip(CASES, got):
        assert g == a.encode("latin-1"), k


def test_rfc6455_known_answer(eng):
    assert eng.encode_keys([b"dGhlIHNhbXBsZSBub25jZQ=="])[0] == b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo=" + b"\0" * 4


def test_block_boundary_lengths_match_host(eng):
    # key + GUID crosses the SHA-1 padding boundaries at key lengths 19/20 and 83/84
    L = libhv_amd.lib()
    L.ws_encode_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    rng = random.Random(3)
    keys = [bytes(rng.randrange(33, 127) for _ in range(n)) for n in list(range(0, 140)) * 3]
    got = eng.encode_keys(keys)
    for k, g in zip(keys, got):
        acc = ctypes.create_string_buffer(32)
        L.ws_encode_key(k, acc)
        assert g == acc.raw, k


def test_large_batch_matches_host(eng):
    L = libhv_amd.lib()
    L.ws_encode_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    rng = random.Random(9)
    keys = [base64.b64encode(rng.randbytes(16)) for _ in range(100000)]
    got = eng.encode_keys(keys)
    for i in range(0, len(keys), 97):
        acc = ctypes.create_string_buffer(32)
        L.ws_encode_key(keys[i], acc)
        assert got[i] == acc.raw


def test_empty_batch(eng):
    assert eng.encode_keys([]) == []
