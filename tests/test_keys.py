"""Handshake digest on the CPU side: the golden
fixture tests/golden/ws_keys.json was produced by the reference ws_encode_key
(http/wsdef.c:11-20, compiled into oracle/_ref); the library's own host
ws_encode_key (libhv_amd/csrc/wsdef.cpp) must reproduce it byte for byte,
including writing exactly 28 bytes (no terminator) into the caller's zeroed
buffer.  The GPU batch is checked against the same fixture in
test_gpu_keys.py."""
from __future__ import annotations

import ctypes
import json
import os

import pytest

import libhv_amd
import wsharness as H

CASES = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ws_keys.json")))["cases"]


def _encode(fn, key: bytes) -> bytes:
    acc = ctypes.create_string_buffer(32)
    fn(key, acc)
    return acc.raw


def test_fixture_shape():
    assert len(CASES) == 2000
    assert sum(len(k) == 24 for k, _ in CASES) >= 1500
    assert all(len(a) == 32 and a.endswith("\0\0\0\0") for _, a in CASES)


def test_rfc6455_known_answer():
    L = libhv_amd.lib()
    L.ws_encode_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    assert _encode(L.ws_encode_key, b"dGhlIHNhbXBsZSBub25jZQ==")[:28] == b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo="


def test_host_ws_encode_key_matches_reference_fixture():
    L = libhv_amd.lib()
    L.ws_encode_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    for k, a in CASES:
        assert _encode(L.ws_encode_key, k.encode()) == a.encode("latin-1"), k


def test_writes_exactly_28_bytes():
    L = libhv_amd.lib()
    L.ws_encode_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    acc = ctypes.create_string_buffer(b"\xaa" * 32, 32)
    L.ws_encode_key(b"dGhlIHNhbXBsZSBub25jZQ==", acc)
    assert acc.raw[28:] == b"\xaa" * 4


@pytest.mark.skipif(not H.have_ref(), reason="reference library not built (GPU box)")
def test_fixture_pinned_to_reference():
    L = H.ref()
    for k, a in CASES[::50]:
        assert _encode(L.ws_encode_key, k.encode()) == a.encode("latin-1")
