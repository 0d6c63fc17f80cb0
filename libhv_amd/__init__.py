"""libhv_amd -- MI355X-native WebSocket server receive path for libhv.

The product is the C-ABI shared library ``libhv_amd/libhvws.so`` (HIP kernels
for gfx950 + C/C++ host code, see include/*.h).  This Python module is a thin
ctypes binding used by the tests and by bench.py; it never computes anything
itself.  Loading fails loudly when the library has not been built: there is
no Python or CPU fallback for the receive path.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# $HVWS_LIB: another build of the library, for A/B runs on one box
LIB_PATH = os.environ.get("HVWS_LIB") or os.path.join(_HERE, "libhvws.so")

# enum websocket_flags (include/websocket_parser.h; reference http/websocket_parser.h:30-45)
WS_OP_CONTINUE, WS_OP_TEXT, WS_OP_BINARY = 0x0, 0x1, 0x2
WS_OP_CLOSE, WS_OP_PING, WS_OP_PONG = 0x8, 0x9, 0xA
WS_FIN, WS_HAS_MASK, WS_OP_MASK = 0x10, 0x20, 0x0F

I_HDR, I_BODY, I_END, I_START = 1 << 10, 1 << 11, 1 << 12, 1 << 13


class WsParser(ctypes.Structure):
    """struct websocket_parser (reference http/websocket_parser.h:50-62), 48 bytes."""

    _fields_ = [
        ("state", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("mask", ctypes.c_char * 4),
        ("mask_offset", ctypes.c_uint8),
        ("length", ctypes.c_size_t),
        ("require", ctypes.c_size_t),
        ("offset", ctypes.c_size_t),
        ("data", ctypes.c_void_p),
    ]

    def fields(self) -> tuple:
        """(state, flags, mask u32, mask_offset, length, require) -- offset excluded (Q12)."""
        return (
            self.state,
            self.flags,
            int.from_bytes(bytes(self.mask), "little"),
            self.mask_offset,
            self.length,
            self.require,
        )


class Segment(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint64)]


class Frame(ctypes.Structure):
    _fields_ = [
        ("hdr_off", ctypes.c_int64),
        ("pay_off", ctypes.c_uint64),
        ("pay_len", ctypes.c_uint64),
        ("length", ctypes.c_uint64),
        ("key", ctypes.c_uint32),
        ("info", ctypes.c_uint32),
    ]


FRAME_DTYPE = np.dtype(
    [("hdr_off", "<i8"), ("pay_off", "<u8"), ("pay_len", "<u8"), ("length", "<u8"), ("key", "<u4"), ("info", "<u4")]
)
assert FRAME_DTYPE.itemsize == ctypes.sizeof(Frame) == 40
assert ctypes.sizeof(WsParser) == 48

MSG_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char), ctypes.c_size_t)

_lib: Optional[ctypes.CDLL] = None

# name -> (restype, argtypes)
_SIGS = {
    "hvws_device_count": (ctypes.c_int, []),
    "hvws_ctx_create": (ctypes.c_void_p, [ctypes.c_int]),
    "hvws_ctx_destroy": (None, [ctypes.c_void_p]),
    "hvws_last_error": (ctypes.c_char_p, []),
    "hvws_ctx_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "hvws_ctx_device": (ctypes.c_int, [ctypes.c_void_p]),
    "hvws_device_identity": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "hvws_dev_alloc": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_dev_free": (None, [ctypes.c_void_p, ctypes.c_void_p]),
    "hvws_host_alloc": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_host_free": (None, [ctypes.c_void_p, ctypes.c_void_p]),
    "hvws_h2d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_d2h": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_d2d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_memset": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64]),
    "hvws_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "hvws_debug_stall": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "hvws_scan": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32],
    ),
    "hvws_unmask": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_step": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32],
    ),
    "hvws_step_resident": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32],
    ),
    "hvws_frame_count": (ctypes.c_int64, [ctypes.c_void_p]),
    "hvws_get_frames": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]),
    "hvws_get_segment_frames": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "hvws_get_carry": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "hvws_last_times": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]),
    "hvws_step_times": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
    "hvws_set_step_event_interval": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "hvws_set_speculation": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hvws_set_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hvws_last_run_repairs": (ctypes.c_int64, [ctypes.c_void_p]),
    "hvws_set_walk_verify": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hvws_last_scan_path": (ctypes.c_int, [ctypes.c_void_p]),
    "hvws_set_fast_bound": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_stream_xor": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]),
    "hvws_rx_batch": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
         ctypes.c_int],
    ),
    "hvws_pipeline": (
        ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    ),
    "hvws_synth": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.POINTER(ctypes.c_uint64)],
    ),
    "hvws_digest": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_build_frames": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
         ctypes.POINTER(ctypes.c_uint64)],
    ),
    "hvws_encode_keys": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p],
    ),
    "hvws_last_kernel_ms": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]),
    "hvws_wsp_new": (ctypes.c_void_p, []),
    "hvws_wsp_free": (None, [ctypes.c_void_p]),
    "hvws_wsp_set_sink": (None, [ctypes.c_void_p, MSG_CB, ctypes.c_void_p]),
    "hvws_wsp_feed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "hvws_wsp_state": (None, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_wsp_feed_many": (
        ctypes.c_int,
        [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
         ctypes.POINTER(ctypes.c_int)],
    ),
    "hvws_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_host_unregister": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "hvws_rx_reads": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p, ctypes.c_uint32,
         ctypes.c_int],
    ),
    "hvws_feeder_new": (ctypes.c_void_p, []),
    "hvws_feeder_free": (None, [ctypes.c_void_p]),
    "hvws_feeder_flush": (ctypes.c_int, [ctypes.c_void_p]),
    "hvws_wsp_feeder_submit": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
         ctypes.c_int, ctypes.POINTER(ctypes.c_int)],
    ),
    "hvws_set_thread_device": (ctypes.c_int, [ctypes.c_int]),
    "hvws_thread_release": (None, []),
    "hvws_unmask_kernel_name": (ctypes.c_char_p, []),
    "hvws_unmask_kernel_name_for": (ctypes.c_char_p, [ctypes.c_uint64]),
    "hvws_run_kernel_name": (ctypes.c_char_p, []),
    "hvws_set_spec_min": (ctypes.c_uint64, [ctypes.c_uint64]),
    "hvws_set_sieve_min": (ctypes.c_uint64, [ctypes.c_uint64]),
    "hvws_set_table_checks": (ctypes.c_int, [ctypes.c_int]),
    "hvws_last_sieve": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_set_sieve_windows": (None, [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_last_sieve_windows": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_build_kernel_name": (ctypes.c_char_p, []),
    "hvws_last_build_kernel": (ctypes.c_char_p, [ctypes.c_void_p]),
    "hvws_last_build_uniform": (ctypes.c_int, [ctypes.c_void_p]),
    "hvws_span_begin": (ctypes.c_int, [ctypes.c_void_p]),
    "hvws_span_end": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]),
    "hvws_set_door": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hvws_debug_dump": (ctypes.c_int, [ctypes.c_int]),
    "hvws_debug_backtraces": (ctypes.c_int, [ctypes.c_int]),
    "hvws_door_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_door_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_door_health": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_set_door_idle_us": (ctypes.c_uint64, [ctypes.c_uint64]),
    "hvws_door_stamps": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "hvws_set_small_batch_limit": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint64]),
    "hvws_set_small_zero_copy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "hvws_set_validation": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_uint32]),
    "hvws_set_unmask_variant": (ctypes.c_int, [ctypes.c_int]),
    # reference ABI (include/websocket_parser.h, include/wsdef.h)
    "websocket_parser_init": (None, [ctypes.c_void_p]),
    "websocket_parser_settings_init": (None, [ctypes.c_void_p]),
    "websocket_parser_execute": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "websocket_parser_decode": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "websocket_decode": (ctypes.c_uint8, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint8]),
    "websocket_calc_frame_size": (ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_size_t]),
    "websocket_build_frame": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "ws_encode_key": (None, [ctypes.c_char_p, ctypes.c_char_p]),
    "ws_calc_frame_size": (ctypes.c_int, [ctypes.c_int, ctypes.c_bool]),
    "ws_build_frame": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_bool, ctypes.c_int, ctypes.c_bool],
    ),
}

# C++ drop-in symbols (include/WebSocketParser.h)
CXX_SYMBOLS = (
    "_Z14hvws_feed_manyPKP15WebSocketParserPKPKcPKmiPi",
    "_Z18hvws_feeder_submitP11hvws_feederPKP15WebSocketParserPKPKcPKmiPi",
    "_ZN15WebSocketParserC1Ev",
    "_ZN15WebSocketParserD1Ev",
    "_ZN15WebSocketParser12FeedRecvDataEPKcm",
)


def lib() -> ctypes.CDLL:
    """Load libhvws.so (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing -- build it with `make -C libhv_amd/csrc` "
            "(or __graft_entry__.build()); the receive path has no CPU fallback"
        )
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class HvwsError(RuntimeError):
    pass


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise HvwsError(f"{what} failed ({rc}): {lib().hvws_last_error().decode(errors='replace')}")


def _ptr(a) -> int:
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a)


class DeviceBuffer:
    def __init__(self, eng: "Engine", nbytes: int):
        self.eng = eng
        self.nbytes = int(nbytes)
        self.ptr = lib().hvws_dev_alloc(eng.ctx, max(self.nbytes, 16))
        if not self.ptr:
            raise HvwsError(f"hvws_dev_alloc({nbytes}): {lib().hvws_last_error().decode()}")

    def free(self) -> None:
        if self.ptr:
            lib().hvws_dev_free(self.eng.ctx, self.ptr)
            self.ptr = None

    def upload(self, arr: np.ndarray, sync: bool = True) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        _check(lib().hvws_h2d(self.eng.ctx, self.ptr, arr.ctypes.data, arr.nbytes), "hvws_h2d")
        if sync:
            self.eng.sync()
        return self

    def download(self, nbytes: Optional[int] = None, dtype=np.uint8) -> np.ndarray:
        n = self.nbytes if nbytes is None else int(nbytes)
        out = np.empty(n, dtype=np.uint8)
        if n:
            _check(lib().hvws_d2h(self.eng.ctx, out.ctypes.data, self.ptr, n), "hvws_d2h")
            self.eng.sync()
        return out.view(dtype)


class Engine:
    """One hvws_ctx (device context + streams + frame tables)."""

    def __init__(self, device: int = 0):
        L = lib()
        self.ctx = L.hvws_ctx_create(device)
        if not self.ctx:
            raise HvwsError(f"hvws_ctx_create({device}): {L.hvws_last_error().decode()}")
        self.device = device

    def close(self) -> None:
        if self.ctx:
            lib().hvws_ctx_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def to_device(self, arr: np.ndarray, pad: int = 64) -> DeviceBuffer:
        arr = np.ascontiguousarray(arr)
        b = DeviceBuffer(self, arr.nbytes + pad)
        if arr.nbytes:
            b.upload(arr)
        return b

    def sync(self) -> None:
        _check(lib().hvws_sync(self.ctx), "hvws_sync")

    @staticmethod
    def _segs(segs: Sequence[Tuple[int, int]]):
        arr = (Segment * max(len(segs), 1))()
        for i, (o, n) in enumerate(segs):
            arr[i].off, arr[i].len = int(o), int(n)
        return arr

    @staticmethod
    def _carry(nseg: int, carry=None):
        arr = (WsParser * max(nseg, 1))()
        for i in range(nseg):
            if carry is not None and carry[i] is not None:
                ctypes.memmove(ctypes.byref(arr[i]), ctypes.byref(carry[i]), ctypes.sizeof(WsParser))
        return arr

    def scan(self, rx: DeviceBuffer, rx_len: int, segs, carry=None) -> int:
        s = self._segs(segs)
        c = self._carry(len(segs), carry)
        _check(lib().hvws_scan(self.ctx, rx.ptr, rx_len, s, c, len(segs)), "hvws_scan")
        return lib().hvws_frame_count(self.ctx)

    def unmask(self, rx: DeviceBuffer, rx_len: int) -> None:
        _check(lib().hvws_unmask(self.ctx, rx.ptr, rx_len), "hvws_unmask")

    def prepare(self, segs, carry=None) -> "Prepared":
        """Build the ctypes segment/carry tables once (for repeated steps)."""
        return Prepared(self._segs(segs), self._carry(len(segs), carry), len(segs))

    def step(self, rx: DeviceBuffer, rx_len: int, segs, carry=None) -> None:
        if isinstance(segs, Prepared):
            s, c, n = segs.segs, segs.carry, segs.n
        else:
            s, c, n = self._segs(segs), self._carry(len(segs), carry), len(segs)
        _check(lib().hvws_step(self.ctx, rx.ptr, rx_len, s, c, n), "hvws_step")

    def step_resident(self, rx: DeviceBuffer, rx_len: int, segs, carry=None) -> None:
        """hvws_step_resident: discovery overlaps the previous step's unmask."""
        if isinstance(segs, Prepared):
            s, c, n = segs.segs, segs.carry, segs.n
        else:
            s, c, n = self._segs(segs), self._carry(len(segs), carry), len(segs)
        _check(lib().hvws_step_resident(self.ctx, rx.ptr, rx_len, s, c, n), "hvws_step_resident")

    def frames(self) -> np.ndarray:
        n = lib().hvws_frame_count(self.ctx)
        out = np.zeros(max(n, 0), dtype=FRAME_DTYPE)
        if n > 0:
            _check(lib().hvws_get_frames(self.ctx, out.ctypes.data, 0, n), "hvws_get_frames")
        return out

    def segment_frames(self, nseg: int) -> Tuple[np.ndarray, np.ndarray]:
        first = np.zeros(nseg, np.uint64)
        cnt = np.zeros(nseg, np.uint64)
        _check(lib().hvws_get_segment_frames(self.ctx, first.ctypes.data, cnt.ctypes.data), "hvws_get_segment_frames")
        return first, cnt

    def carry(self, nseg: int):
        arr = (WsParser * max(nseg, 1))()
        started = (ctypes.c_int * max(nseg, 1))()
        _check(lib().hvws_get_carry(self.ctx, arr, started), "hvws_get_carry")
        return [arr[i] for i in range(nseg)], [started[i] for i in range(nseg)]

    def last_times(self) -> Tuple[float, float]:
        out = (ctypes.c_float * 2)()
        _check(lib().hvws_last_times(self.ctx, out), "hvws_last_times")
        return float(out[0]), float(out[1])

    def step_times(self, max_steps: int = 32) -> List[Tuple[float, float]]:
        """(scan ms, unmask ms) of the last max_steps steps (at most 32), oldest first."""
        out = (ctypes.c_float * (2 * max_steps))()
        n = lib().hvws_step_times(self.ctx, out, max_steps)
        if n < 0:
            _check(n, "hvws_step_times")
        return [(float(out[2 * i]), float(out[2 * i + 1])) for i in range(n)]

    def set_step_event_interval(self, every: int) -> int:
        """Timing events on every `every`-th step only (hvws_set_step_event_interval); returns the old interval."""
        r = lib().hvws_set_step_event_interval(self.ctx, every)
        if r < 0:
            _check(r, "hvws_set_step_event_interval")
        return r

    def stream_xor(self, buf: DeviceBuffer, n: int, pattern: int) -> None:
        _check(lib().hvws_stream_xor(self.ctx, buf.ptr, n, pattern), "hvws_stream_xor")

    def rx_batch(self, host: np.ndarray, segs, carry=None, unmask: bool = True):
        s = self._segs(segs)
        c = self._carry(len(segs), carry)
        _check(lib().hvws_rx_batch(self.ctx, host.ctypes.data, host.nbytes, s, c, len(segs), int(unmask)),
               "hvws_rx_batch")
        return [c[i] for i in range(len(segs))]

    def synth(self, buf: DeviceBuffer, buf_len: int, seed: int, plan: "DevicePlan", mode: int = 0) -> int:
        bad = ctypes.c_uint64(0)
        _check(
            lib().hvws_synth(self.ctx, buf.ptr, buf_len, seed, plan.n, plan.off.ptr, plan.flags.ptr, plan.mask.ptr,
                             plan.length.ptr, plan.text.ptr if plan.text else None, mode, ctypes.byref(bad)),
            "hvws_synth",
        )
        return int(bad.value)

    def build_frames(self, out: DeviceBuffer, out_cap: int, payload: Optional[DeviceBuffer], payload_len: int,
                     tx: "TxPlan", out_off: Optional[DeviceBuffer] = None) -> int:
        """Transmit side: websocket_build_frame for every frame of `tx` into
        `out` (back to back).  Returns the bytes written (the kernel runs
        asynchronously on the ctx stream)."""
        n = ctypes.c_uint64(0)
        _check(
            lib().hvws_build_frames(self.ctx, out.ptr, out_cap, payload.ptr if payload else None, payload_len,
                                    tx.pay_off.ptr, tx.length.ptr, tx.flags.ptr, tx.mask.ptr if tx.mask else None,
                                    tx.n, out_off.ptr if out_off else None, ctypes.byref(n)),
            "hvws_build_frames",
        )
        return int(n.value)

    def encode_keys(self, keys: Sequence[bytes]) -> List[bytes]:
        """Sec-WebSocket-Accept for every key (ws_encode_key, batched on the GPU)."""
        n = len(keys)
        if n == 0:
            return []
        lens = np.array([len(k) for k in keys], dtype=np.uint32)
        offs = np.zeros(n, dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        blob = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8)
        dk, do, dl = self.to_device(blob), self.to_device(offs), self.to_device(lens)
        acc = self.alloc(32 * n)
        try:
            _check(lib().hvws_encode_keys(self.ctx, dk.ptr, do.ptr, dl.ptr, n, acc.ptr), "hvws_encode_keys")
            raw = acc.download(32 * n).tobytes()
        finally:
            for b in (dk, do, dl, acc):
                b.free()
        return [raw[32 * i:32 * i + 32] for i in range(n)]

    def last_kernel_ms(self) -> float:
        out = ctypes.c_float(0)
        _check(lib().hvws_last_kernel_ms(self.ctx, ctypes.byref(out)), "hvws_last_kernel_ms")
        return float(out.value)

    def digest(self, buf: DeviceBuffer, n: int) -> int:
        out = ctypes.c_uint64(0)
        _check(lib().hvws_digest(self.ctx, buf.ptr, n, ctypes.byref(out)), "hvws_digest")
        return int(out.value)


class Prepared:
    def __init__(self, segs, carry, n):
        self.segs, self.carry, self.n = segs, carry, n


class DevicePlan:
    """A synthetic batch plan resident on the device (see libhv_amd.synth)."""

    def __init__(self, eng: Engine, plan):
        self.n = len(plan.length)
        self.off = eng.to_device(plan.frame_off.astype(np.uint64))
        self.flags = eng.to_device(plan.flags.astype(np.uint8))
        self.mask = eng.to_device(plan.mask.astype(np.uint32))
        self.length = eng.to_device(plan.length.astype(np.uint64))
        self.text = eng.to_device(plan.text.astype(np.uint8)) if plan.text is not None else None

    def free(self):
        for b in (self.off, self.flags, self.mask, self.length, self.text):
            if b is not None:
                b.free()


class TxPlan:
    """Outgoing-frame tables on the device for Engine.build_frames: frame i is
    websocket_build_frame(flags[i], mask[i], payload + pay_off[i], length[i])."""

    def __init__(self, eng: Engine, pay_off, length, flags, mask=None):
        self.n = len(length)
        self.pay_off = eng.to_device(np.asarray(pay_off, dtype=np.uint64))
        self.length = eng.to_device(np.asarray(length, dtype=np.uint64))
        self.flags = eng.to_device(np.asarray(flags, dtype=np.uint8))
        self.mask = eng.to_device(np.asarray(mask, dtype=np.uint32)) if mask is not None else None

    def free(self):
        for b in (self.pay_off, self.length, self.flags, self.mask):
            if b is not None:
                b.free()


def device_count() -> int:
    return lib().hvws_device_count()


def device_identity(device: int) -> tuple:
    """(PCI bus id, the device hipGetDevice reports once `device` is
    selected): which physical card a rank ran on."""
    buf = ctypes.create_string_buffer(64)
    cur = ctypes.c_int(-1)
    _check(lib().hvws_device_identity(device, buf, 64, ctypes.byref(cur)), "hvws_device_identity")
    return buf.value.decode(), int(cur.value)

