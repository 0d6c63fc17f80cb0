#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE.

Run in the build container, where /root/reference exists and
`make -C oracle` has compiled libhv's own http/websocket_parser.c,
http/wsdef.c, util/sha1.c and util/base64.c into oracle/_ref/libwsref.so.
Every expected output below comes from that library:
  * frames are built with the reference's websocket_build_frame;
  * callback logs come from the reference's websocket_parser_execute
    (driven by tests/csrc/evlog.c), with the reference's
    websocket_parser_decode when `decode` is set;
  * message logs come from oracle/ws_msg.cpp compiled against the reference
    frame parser (the restated WebSocketParser.cpp, see oracle/Makefile);
  * config digests hash reference-built batches and their reference-unmasked
    form.
The fixtures are data (inputs + expected outputs); no reference source is
stored.  Usage: python tests/golden/make_golden.py [--configs c1,c2,c4]
       python tests/golden/make_golden.py --skip-streams --configs '' \\
              --big c3,c5_rank0,c5_rank1,c5_rank2,c5_rank3,c5_rank4,c5_rank5,c5_rank6,c5_rank7
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import random
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import streams as S  # noqa: E402
import wsharness as H  # noqa: E402
from libhv_amd import synth  # noqa: E402


def ser_msgs(res) -> bytes:
    msgs, rets, state, buf = res
    out = bytearray()
    out += struct.pack("<I", len(msgs))
    for op, b in msgs:
        out += struct.pack("<iQ", op, len(b)) + b
    out += struct.pack("<I", len(rets)) + struct.pack(f"<{len(rets)}i", *rets)
    out += struct.pack("<8Q", *state)
    return bytes(out)


def stream_cases():
    rng = random.Random(20261015)
    cases = []
    for name, data in S.quirk_streams():
        modes = ["one", "small", "bytes"] if len(data) <= 2048 else ["one", "rand"]
        for mode in modes:
            for decode in (False, True):
                chunks = S.rand_chunks(random.Random(len(cases)), len(data), mode)
                cases.append(dict(name=f"{name}/{mode}/{'dec' if decode else 'raw'}", data=data, chunks=chunks,
                                  abort_at=-1, decode=decode))
    for t in range(48):
        data = S.rand_stream(rng, rng.randint(1, 12), max_len=rng.choice([30, 300, 3000]))
        mode = rng.choice(["one", "rand", "small"])
        chunks = S.rand_chunks(rng, len(data), mode)
        abort_at = rng.choice([-1, -1, rng.randint(0, 12)])
        cases.append(dict(name=f"random{t}/{mode}", data=data, chunks=chunks, abort_at=abort_at,
                          decode=rng.random() < 0.5))
    return cases


def make_streams():
    assert H.have_ref(), "oracle/_ref/libwsref.so missing: run `make -C oracle` where /root/reference exists"
    arrays = {}
    meta = []
    for i, c in enumerate(stream_cases()):
        log, buf = H.run_evlog("ref", c["data"], c["chunks"], c["abort_at"], c["decode"])
        msgs = H.run_messages("ref", c["data"], c["chunks"])
        arrays[f"in{i}"] = np.frombuffer(c["data"], np.uint8)
        arrays[f"chunks{i}"] = np.array(c["chunks"], np.uint64)
        arrays[f"log{i}"] = np.frombuffer(log, np.uint8)
        arrays[f"buf{i}"] = np.frombuffer(buf, np.uint8)
        arrays[f"msgs{i}"] = np.frombuffer(ser_msgs(msgs), np.uint8)
        arrays[f"mbuf{i}"] = np.frombuffer(msgs[3], np.uint8)
        meta.append(dict(name=c["name"], abort_at=c["abort_at"], decode=c["decode"]))
    np.savez_compressed(os.path.join(HERE, "streams.npz"), **arrays)
    with open(os.path.join(HERE, "streams.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "source": "oracle/_ref/libwsref.so (reference C)",
                   "cases": meta}, f, indent=1)
    print(f"streams: {len(meta)} cases")


def make_kat():
    L = H.ref()
    acc = ctypes.create_string_buffer(64)
    L.ws_encode_key(b"dGhlIHNhbXBsZSBub25jZQ==", acc)
    kat = {"ws_encode_key": {"dGhlIHNhbXBsZSBub25jZQ==": acc.value.decode()}}
    frames = []
    rng = random.Random(7)
    for n in S.EDGE_LENS + [1000, 70000]:
        for fl in (0x1 | 0x10 | 0x20, 0x2 | 0x20, 0x9 | 0x10, 0x0, 0xA | 0x10 | 0x20):
            data = rng.randbytes(n)
            key = rng.randbytes(4)
            out = H.build_frames_ref([(fl, data, key)])
            frames.append({"flags": fl, "len": n, "data_sha256": hashlib.sha256(data).hexdigest(),
                           "seed_bytes": None, "key": key.hex(), "frame_sha256": hashlib.sha256(out).hexdigest(),
                           "frame_head": out[:24].hex()})
    kat["build_frame"] = {"rng": "random.Random(7).randbytes per (len, flags) in order", "cases": frames}
    b = ctypes.create_string_buffer(16)
    n = L.ws_build_frame(b, b"Hello", 5, bytes.fromhex("37fa213d"), True, 1, True)
    kat["rfc6455_hello_masked"] = b.raw[:n].hex()
    n = L.ws_build_frame(b, b"Hello", 5, None, False, 1, True)
    kat["rfc6455_hello_unmasked"] = b.raw[:n].hex()
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    print("kat written")


def make_keys():
    """Sec-WebSocket-Accept for 1500 conforming keys (base64 of a 16-byte
    nonce) and 500 keys of other lengths (0-200 printable bytes), from the
    reference ws_encode_key."""
    import base64
    L = H.ref()
    rng = random.Random(4455)
    keys = [base64.b64encode(rng.randbytes(16)) for _ in range(1500)]
    keys += [bytes(rng.randrange(33, 127) for _ in range(rng.randrange(0, 201))) for _ in range(500)]
    out = []
    for k in keys:
        acc = ctypes.create_string_buffer(32)
        L.ws_encode_key(k, acc)
        out.append([k.decode(), acc.raw.decode("latin-1")])
    with open(os.path.join(HERE, "ws_keys.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py make_keys", "source": "oracle/_ref/libwsref.so "
                   "ws_encode_key into zeroed char[32]", "cases": out}, f, indent=0)
    print(f"ws_keys: {len(out)} cases")


def ref_build(plan) -> np.ndarray:
    """Batch built frame by frame by the reference websocket_build_frame."""
    L = H.ref()
    O = H.oracle()
    buf = np.zeros(plan.total, dtype=np.uint8)
    base = buf.ctypes.data
    maxlen = int(plan.length.max()) if plan.n else 0
    tmp = ctypes.create_string_buffer(max(maxlen, 1))
    for i in range(plan.n):
        n = int(plan.length[i])
        O.ows_synth_plain(tmp, plan.seed, i, n, int(plan.text[i]) if plan.text is not None else 0)
        key = int(plan.mask[i]).to_bytes(4, "little")
        L.websocket_build_frame(base + int(plan.frame_off[i]), int(plan.flags[i]), key, tmp, n)
    return buf


def make_configs(names):
    path = os.path.join(HERE, "configs.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name in names:
        plan = synth.config_plan(name, seed=1)
        buf = ref_build(plan)
        assert np.array_equal(buf, H.synth_cpu(plan)), "oracle generator != reference websocket_build_frame"
        d_masked = H.digest_np(buf)
        sha_in = hashlib.sha256(buf.tobytes()).hexdigest()
        # unmask through the reference frame parser + restated WebSocketParser, 8 KiB chunks
        stats = (ctypes.c_uint64 * 4)()
        rc = H.ref().msgp_bench_feed(buf.ctypes.data, buf.nbytes, 8192, stats)
        assert rc == 0
        d_plain = H.digest_np(buf)
        out[name] = {
            "plan": {"fn": f"libhv_amd.synth.config_plan('{name}', seed=1)", "frames": plan.n, "rx_bytes": plan.total,
                     "payload_bytes": plan.payload_bytes},
            "digest_masked": f"{d_masked:016x}",
            "digest_unmasked": f"{d_plain:016x}",
            "sha256_masked": sha_in,
            "sha256_unmasked": hashlib.sha256(buf.tobytes()).hexdigest(),
            "messages": int(stats[0]),
            "message_bytes": int(stats[1]),
            "message_xsum": int(stats[2]),
            "chunk": 8192,
        }
        print(name, out[name]["frames"] if "frames" in out[name] else plan.n, "ok")
        del buf
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


def big_plan(name: str):
    """c3 (seed 1, the tests' batch) or c5_rank{r}: the c3-shaped batch bench.py
    rank r builds (synth.config_plan('c3', seed=1000 + r))."""
    if name == "c3":
        return synth.config_plan("c3", seed=1)
    if name.startswith("c5_rank"):
        return synth.config_plan("c3", seed=1000 + int(name[len("c5_rank"):]))
    raise KeyError(name)


def streamed_digest(plan, threads: int):
    return H.streamed_digest(plan, threads, "ref")


def make_big_configs(names, threads: int):
    """Configs too large to hold (c3: 68.7 GB; the eight config-5 rank
    batches): reference digests streamed in bounded memory.  Checked first on
    c2, whose whole-buffer digests (make_configs) are committed."""
    path = os.path.join(HERE, "configs.json")
    out = json.load(open(path))
    d = streamed_digest(synth.config_plan("c2", seed=1), threads)
    g = out["c2"]
    assert (f"{d[0]:016x}", f"{d[1]:016x}", d[2], d[3], d[4]) == (
        g["digest_masked"], g["digest_unmasked"], g["messages"], g["message_bytes"], g["message_xsum"]), \
        "streamed digest != whole-buffer digest on c2"
    for name in names:
        plan = big_plan(name)
        d = streamed_digest(plan, threads)
        fn = "config_plan('c3', seed=1)" if name == "c3" else f"config_plan('c3', seed={plan.seed})"
        out[name] = {
            "plan": {"fn": f"libhv_amd.synth.{fn}", "frames": plan.n, "rx_bytes": plan.total,
                     "payload_bytes": plan.payload_bytes},
            "digest_masked": f"{d[0]:016x}",
            "digest_unmasked": f"{d[1]:016x}",
            "messages": d[2],
            "message_bytes": d[3],
            "message_xsum": d[4],
            "chunk": 8192,
            "method": "streamed: reference websocket_build_frame per frame + reference parser in 8 KiB chunks, "
                      "digest folded per 8-byte word (tests/csrc/cfgdigest.c)",
        }
        print(name, plan.n, out[name]["digest_masked"], out[name]["digest_unmasked"], flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2")
    ap.add_argument("--big", default="", help="streamed digests, e.g. c3,c5_rank0,...,c5_rank7")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--skip-streams", action="store_true")
    ap.add_argument("--only-keys", action="store_true")
    a = ap.parse_args()
    if a.only_keys:
        make_keys()
        return
    if not a.skip_streams:
        make_kat()
        make_keys()
        make_streams()
    if a.configs:
        make_configs([c for c in a.configs.split(",") if c])
    if a.big:
        make_big_configs([c for c in a.big.split(",") if c], a.threads)


if __name__ == "__main__":
    main()
