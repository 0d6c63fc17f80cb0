"""Test harness: ctypes access to the CPU oracle (oracle/), the compiled
reference (oracle/_ref/, present only where /root/reference was), the
callback-log driver (tests/csrc/evlog.c) and the product (libhv_amd).

Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() use the
oracle; the product never does.
"""
from __future__ import annotations

import ctypes
import os
import struct
from typing import List, Optional, Sequence, Tuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libwsoracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libwsref.so")
EVLOG_SO = os.path.join(ROOT, "tests", "_build", "libevlog.so")

_cache = {}

MSG_SINK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char), ctypes.c_size_t)


class OFrame(ctypes.Structure):
    _fields_ = [
        ("hdr_off", ctypes.c_int64),
        ("pay_off", ctypes.c_uint64),
        ("pay_len", ctypes.c_uint64),
        ("length", ctypes.c_uint64),
        ("key", ctypes.c_uint32),
        ("info", ctypes.c_uint32),
    ]


def _load(path: str, kind: str) -> ctypes.CDLL:
    if path in _cache:
        return _cache[path]
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing (run __graft_entry__.build())")
    L = ctypes.CDLL(path)
    if kind in ("oracle", "ref"):
        L.msgp_new.restype = ctypes.c_void_p
        L.msgp_free.argtypes = [ctypes.c_void_p]
        L.msgp_set_sink.argtypes = [ctypes.c_void_p, MSG_SINK, ctypes.c_void_p]
        L.msgp_feed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.msgp_feed.restype = ctypes.c_int
        L.msgp_state.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        L.msgp_bench_feed.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)]
        L.msgp_bench_feed.restype = ctypes.c_int
        L.msgp_bench_decode_spans.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_size_t]
        L.msgp_bench_decode_spans.restype = ctypes.c_uint64
    if kind == "oracle":
        L.ows_scan_segment.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
        L.ows_scan_segment.restype = ctypes.c_size_t
        L.ows_synth_fill.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p]
        L.ows_synth_plain.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]
        L.ows_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint8]
        L.ows_decode.restype = ctypes.c_uint8
        L.ows_build_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_size_t]
        L.ows_build_frame.restype = ctypes.c_size_t
        L.ows_calc_frame_size.argtypes = [ctypes.c_uint32, ctypes.c_size_t]
        L.ows_calc_frame_size.restype = ctypes.c_size_t
        L.ows_fnv1a.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
        L.ows_fnv1a.restype = ctypes.c_uint64
        L.ows_ws_build_frame.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ows_ws_build_frame.restype = ctypes.c_int
    if kind == "ref":
        L.websocket_build_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_size_t]
        L.websocket_build_frame.restype = ctypes.c_size_t
        L.ws_encode_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.ws_build_frame.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_bool, ctypes.c_int, ctypes.c_bool]
        L.ws_build_frame.restype = ctypes.c_int
    if kind == "evlog":
        L.evlog_feed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64,
                                 ctypes.c_void_p, ctypes.c_size_t]
        L.evlog_feed.restype = ctypes.c_int64
    _cache[path] = L
    return L


def oracle() -> ctypes.CDLL:
    return _load(ORACLE_SO, "oracle")


def have_ref() -> bool:
    return os.path.exists(REF_SO)


def ref() -> ctypes.CDLL:
    return _load(REF_SO, "ref")


def evlog() -> ctypes.CDLL:
    return _load(EVLOG_SO, "evlog")


def product() -> ctypes.CDLL:
    import libhv_amd

    return libhv_amd.lib()


def _addr(L: ctypes.CDLL, name: str) -> int:
    return ctypes.cast(getattr(L, name), ctypes.c_void_p).value


def exec_fns(impl: str) -> Tuple[int, int, int]:
    """(execute, init, parser_decode) function addresses of an implementation."""
    if impl == "oracle":
        L = oracle()
        return _addr(L, "ows_execute"), _addr(L, "ows_parser_init"), _addr(L, "ows_parser_decode")
    if impl == "ref":
        L = ref()
    elif impl == "gpu":
        L = product()
    else:
        raise KeyError(impl)
    return (_addr(L, "websocket_parser_execute"), _addr(L, "websocket_parser_init"),
            _addr(L, "websocket_parser_decode"))


def run_evlog(impl: str, data: bytes, chunks: Sequence[int], abort_at: int = -1,
              decode: bool = False) -> Tuple[bytes, bytes]:
    """Feed data through impl's websocket_parser_execute in the given chunk
    sizes; return (callback log, buffer after the run)."""
    ex, init, dec = exec_fns(impl)
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    ch = (ctypes.c_uint64 * max(len(chunks), 1))(*chunks)
    cap = 64 * (len(data) + 16) * 8 + 4096
    log = ctypes.create_string_buffer(cap)
    n = evlog().evlog_feed(ex, init, dec if decode else None, buf, len(data), ch, len(chunks), abort_at, log, cap)
    if n < 0:
        raise RuntimeError("evlog overflow")
    return log.raw[:n], buf.raw[: len(data)]


class MsgLog:
    def __init__(self):
        self.msgs: List[Tuple[int, bytes]] = []
        self.cb = MSG_SINK(self._on)

    def _on(self, user, opcode, data, n):
        self.msgs.append((int(opcode), ctypes.string_at(data, n) if n else b""))


def run_messages(impl: str, data: bytes, chunks: Sequence[int]):
    """Feed through the message layer (WebSocketParser semantics).  Returns
    (messages, per-call return values, final state[8], buffer after)."""
    sink = MsgLog()
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    st = (ctypes.c_uint64 * 8)()
    rets = []
    if impl in ("oracle", "ref"):
        L = oracle() if impl == "oracle" else ref()
        h = L.msgp_new()
        L.msgp_set_sink(h, sink.cb, None)
        feed = lambda p, n: L.msgp_feed(h, p, n)
        state = lambda: L.msgp_state(h, st)
        free = lambda: L.msgp_free(h)
    else:
        import libhv_amd

        L = libhv_amd.lib()
        h = L.hvws_wsp_new()
        sink.gpu_cb = libhv_amd.MSG_CB(sink._on)   # keep the thunk alive while the handle may call it
        L.hvws_wsp_set_sink(h, sink.gpu_cb, None)
        feed = lambda p, n: L.hvws_wsp_feed(h, p, n)
        state = lambda: L.hvws_wsp_state(h, st)
        free = lambda: L.hvws_wsp_free(h)
    base = ctypes.addressof(buf)
    at = 0
    for n in chunks:
        if at >= len(data):
            break
        n = min(n, len(data) - at)
        rets.append(feed(base + at, n))
        at += n
    state()
    free()
    return sink.msgs, rets, tuple(st), buf.raw[: len(data)]


def scan_segment(data: bytes, carry: Optional[ctypes.Structure] = None, cap: Optional[int] = None):
    """Oracle frame records for one segment (WebSocketParser semantics).
    Returns (records ndarray, carry-out parser, started, unmasked buffer)."""
    import libhv_amd

    L = oracle()
    st = libhv_amd.WsParser()
    if carry is not None:
        ctypes.memmove(ctypes.byref(st), ctypes.byref(carry), ctypes.sizeof(st))
    else:
        L.ows_parser_init(ctypes.byref(st))
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    cap = cap if cap is not None else len(data) // 2 + 4
    recs = (OFrame * max(cap, 1))()
    started = ctypes.c_int(0)
    n = L.ows_scan_segment(ctypes.byref(st), buf, len(data), recs, cap, ctypes.byref(started))
    assert n <= cap
    arr = np.frombuffer(bytes(recs)[: n * ctypes.sizeof(OFrame)], dtype=libhv_amd.FRAME_DTYPE).copy()
    return arr, st, started.value, buf.raw[: len(data)]


def synth_cpu(plan, seed: Optional[int] = None) -> np.ndarray:
    """Oracle build of a plan's batch (websocket_build_frame layout)."""
    L = oracle()
    buf = np.zeros(plan.total, dtype=np.uint8)
    off = np.ascontiguousarray(plan.frame_off, dtype=np.uint64)
    fl = np.ascontiguousarray(plan.flags, dtype=np.uint8)
    mk = np.ascontiguousarray(plan.mask, dtype=np.uint32)
    ln = np.ascontiguousarray(plan.length, dtype=np.uint64)
    tx = np.ascontiguousarray(plan.text, dtype=np.uint8) if plan.text is not None else None
    L.ows_synth_fill(buf.ctypes.data, buf.nbytes, plan.seed if seed is None else seed, plan.n, off.ctypes.data,
                     fl.ctypes.data, mk.ctypes.data, ln.ctypes.data, tx.ctypes.data if tx is not None else None)
    return buf


def build_frames_ref(frames: Sequence[Tuple[int, bytes, Optional[bytes]]]) -> bytes:
    """Concatenate frames built by the reference websocket_build_frame
    (flags, payload, key or None) -- falls back to the oracle when the
    reference library is not present."""
    use_ref = have_ref()
    L = ref() if use_ref else oracle()
    fn = L.websocket_build_frame if use_ref else L.ows_build_frame
    out = bytearray()
    for flags, payload, key in frames:
        buf = ctypes.create_string_buffer(len(payload) + 16)
        k = ctypes.create_string_buffer(key, 4) if key is not None else None
        n = fn(buf, flags, k, payload, len(payload))
        out += buf.raw[:n]
    return bytes(out)


def parse_log(log: bytes) -> list:
    """Decode an evlog byte log into tuples (for readable diffs)."""
    out = []
    i = 0
    while i < len(log):
        t = chr(log[i])
        i += 1
        if t == "H":
            out.append(("H",) + struct.unpack_from("<IIQQIB", log, i))
            i += 4 + 4 + 8 + 8 + 4 + 1
        elif t == "B":
            out.append(("B",) + struct.unpack_from("<QQIQIB", log, i))
            i += 8 + 8 + 4 + 8 + 4 + 1
        elif t == "E":
            out.append(("E",) + struct.unpack_from("<IQIB", log, i))
            i += 4 + 8 + 4 + 1
        elif t == "R":
            out.append(("R",) + struct.unpack_from("<QIIIBQQ", log, i))
            i += 8 + 4 + 4 + 4 + 1 + 8 + 8
        else:
            raise ValueError(f"bad tag {t!r} at {i - 1}")
    return out


def digest_np(buf: np.ndarray) -> int:
    """Host restatement of hvws_digest (include/hvws_synth.h)."""
    from libhv_amd.synth import mix64

    b = np.asarray(buf, dtype=np.uint8)
    pad = (-len(b)) % 8
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    w = b.view("<u8")
    k = np.arange(len(w), dtype=np.uint64) * np.uint64(0xD1B54A32D192ED03)
    return int(mix64(w ^ k).sum(dtype=np.uint64))


class _CfgFns(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in ("build", "mnew", "msink", "mfeed", "mfree", "synth")]


CFGDIGEST_SO = os.path.join(ROOT, "tests", "_build", "libcfgdigest.so")


def streamed_digest(plan, threads: int, impl: str = "ref"):
    """[digest_masked, digest_unmasked, messages, message_bytes, message_xsum]
    of a plan's batch without holding it (tests/csrc/cfgdigest.c): frames built
    window by window by `impl`'s websocket_build_frame ("ref": the reference's,
    oracle/_ref; "oracle": the restatement), unmasked by its parser + message
    layer in 8 KiB chunks.  Plans with fragments run as one range."""
    L, O = (ref() if impl == "ref" else oracle()), oracle()
    D = _load(CFGDIGEST_SO, "cfgdigest")
    fin_only = bool(np.all((plan.flags & 0x10) != 0) and np.all((plan.flags & 0x0F) != 0))
    if not fin_only:
        threads = 1   # fragments carry message state across frames: one range
    build = "websocket_build_frame" if impl == "ref" else "ows_build_frame"
    fns = _CfgFns(_addr(L, build), _addr(L, "msgp_new"), _addr(L, "msgp_set_sink"), _addr(L, "msgp_feed"),
                  _addr(L, "msgp_free"), _addr(O, "ows_synth_plain"))
    off = np.ascontiguousarray(plan.frame_off, np.uint64)
    fl = np.ascontiguousarray(plan.flags, np.uint8)
    mk = np.ascontiguousarray(plan.mask, np.uint32)
    ln = np.ascontiguousarray(plan.length, np.uint64)
    tx = np.ascontiguousarray(plan.text, np.uint8) if plan.text is not None else None
    out = (ctypes.c_uint64 * 5)()
    D.cfgd_run.restype = ctypes.c_int
    D.cfgd_run.argtypes = [ctypes.POINTER(_CfgFns), ctypes.c_uint64, ctypes.c_uint64] + [ctypes.c_void_p] * 5 + \
        [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    rc = D.cfgd_run(ctypes.byref(fns), plan.seed, plan.n, off.ctypes.data, fl.ctypes.data, mk.ctypes.data,
                    ln.ctypes.data, tx.ctypes.data if tx is not None else None, plan.total, threads, out)
    assert rc == 0, "cfgd_run failed"
    return [int(x) for x in out]
