"""CPU: the RFC 6455 validation oracle (tests/wsvalidate.py) is
self-consistent -- the classes its frame generator intends are the classes
its stream walker derives from the bytes -- and frames it calls valid parse
through the reference restatement unchanged.  GPU checks: test_gpu_validate.py."""
from __future__ import annotations

import random

import wsharness as H
import wsvalidate as V


def test_generator_matches_walker():
    for seed in range(200):
        data, exp = V.random_stream(seed, 200, tail_len64=seed % 2 == 0)
        assert [v for _, v in V.violations(data)] == exp


def test_every_class_is_generated():
    seen = 0
    for seed in range(50):
        _, exp = V.random_stream(seed, 200, tail_len64=True)
        for v in exp:
            seen |= v
    assert seen == V.V_ALL


def test_known_headers():
    assert V.violations(bytes([0x81, 0x80, 1, 2, 3, 4])) == [(0, 0)]                  # masked empty TEXT
    assert V.violations(bytes([0xC1, 0x80, 1, 2, 3, 4])) == [(0, V.V_RSV)]            # RSV1
    assert V.violations(bytes([0x83, 0x80, 1, 2, 3, 4])) == [(0, V.V_OPCODE)]         # opcode 3
    assert V.violations(bytes([0x09, 0x80, 1, 2, 3, 4])) == [(0, V.V_CONTROL)]        # fragmented PING
    assert V.violations(bytes([0x81, 0x00])) == [(0, V.V_UNMASKED)]                   # unmasked
    assert V.violations(bytes([0x82, 0xFE, 0, 5, 1, 2, 3, 4]) + b"x" * 5) == [(0, V.V_NONMIN)]


def test_reference_accepts_what_validation_flags():
    """The reference validates nothing: the oracle parses every
    generated stream to the end, callbacks and all."""
    rng = random.Random(1)
    for seed in range(5):
        data, _ = V.random_stream(seed, 100)
        log, _ = H.run_evlog("oracle", data, [rng.randrange(1, 4000) for _ in range(len(data))])
        assert log
