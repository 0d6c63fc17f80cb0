"""Child process of test_gpu_door.py::test_door_request_in_pinned_host_memory
(not a test module): with $HVWS_EXPERIMENT door_vram=0 the worker's request
block and bytes live in pinned host memory -- the layout a box without a
large BAR gets -- and the worker polls them across PCIe.  Feeds, decodes and
masked builds through the worker are checked against the oracle; prints
"ok <requests>" and exits 0, or raises."""
import ctypes
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import libhv_amd  # noqa: E402
import streams as S  # noqa: E402
import wsharness as H  # noqa: E402

L = libhv_amd.lib()
L.hvws_set_door(None, 1)
rng = random.Random(23)
for _ in range(30):
    data = S.rand_stream(rng, rng.randint(1, 14), max_len=rng.choice([30, 300, 3000, 9000]))
    chunks = S.rand_chunks(rng, len(data), rng.choice(["rand", "small", "one"]))
    assert H.run_messages("gpu", data, chunks) == H.run_messages("oracle", data, chunks)
O = H.oracle()
for n in (0, 1, 5, 125, 4097, 32768):
    src = rng.randbytes(n)
    key = rng.randbytes(4)
    a = ctypes.create_string_buffer(n + 1)
    b = ctypes.create_string_buffer(n + 1)
    assert L.websocket_decode(a, src, n, key, 1) == O.ows_decode(b, src, n, key, 1) and a.raw[:n] == b.raw[:n]
    out = ctypes.create_string_buffer(n + 16)
    m = L.websocket_build_frame(out, 0x2 | 0x20, key, src, n)
    assert out.raw[:m] == H.build_frames_ref([(0x2 | 0x20, src, key)])
info = (ctypes.c_uint64 * 2)()
L.hvws_door_info(None, info)
assert info[0] == 0, "the request area is in device memory despite door_vram=0"
st = (ctypes.c_uint64 * 4)()
L.hvws_door_stats(None, st)
assert st[1] > 0, "no request reached the worker"
h = (ctypes.c_uint64 * 2)()
L.hvws_door_health(h)
assert (h[0], h[1]) == (0, 0), "a worker wedged or a request went unanswered"
L.hvws_thread_release()
print("ok", int(st[1]), flush=True)
