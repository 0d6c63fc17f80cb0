"""Where a FeedRecvData read spends its time on the resident worker: device
stamps (100 MHz realtime clock) of each 8 KiB read -- request seen -> staged
-> walked -> XORed -> records written -- against the host's wall time per
call.  Medians over n reads."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the worker writes its phase stamps only when asked ($HVWS_EXPERIMENT door_stamps=1)
os.environ["HVWS_EXPERIMENT"] = ",".join(x for x in (os.environ.get("HVWS_EXPERIMENT", ""), "door_stamps=1") if x)
sys.path.insert(0, ROOT)
import libhv_amd  # noqa: E402
from libhv_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
L = libhv_amd.lib()
with libhv_amd.Engine(0) as eng:
    fp = synth.uniform_plan(n * 8 + 16, 1024, 5)
    dp = libhv_amd.DevicePlan(eng, fp)
    b = eng.alloc(fp.total + 64)
    eng.synth(b, fp.total, fp.seed, dp, 0)
    data = b.download(fp.total)
    b.free()
    dp.free()
buf = ctypes.create_string_buffer(data.tobytes(), len(data))
# DOOR_PHASES_BUSY=1: another context keeps the GPU busy with short kernels
# meanwhile (does the worker's single workgroup run slower on an idle chip?)
busy = os.environ.get("DOOR_PHASES_BUSY") == "1"
stop = []
if busy:
    import threading

    def keep_busy():
        with libhv_amd.Engine(0) as e2:
            bb = e2.alloc(1 << 20)
            while not stop:
                e2.stream_xor(bb, 1 << 20, 0x5A5A5A5A)
                e2.sync()
            bb.free()

    th = threading.Thread(target=keep_busy, daemon=True)
    th.start()
    time.sleep(0.5)
L.hvws_set_door(None, 1)
h = L.hvws_wsp_new()
st = (ctypes.c_uint64 * 12)()
rows, wall = [], []
for i in range(n):
    t = time.perf_counter()
    r = L.hvws_wsp_feed(h, ctypes.addressof(buf) + i * 8192, 8192)
    wall.append(time.perf_counter() - t)
    assert r == 8192
    L.hvws_door_stamps(None, st)
    rows.append(list(st[:12]))
if busy:
    stop.append(1)
    th.join()
rows = np.array(rows[n // 10:], dtype=np.float64)
t0, t1, t2, t3, t4, t5, rel, tw, tc, tp, tt, tx = (rows[:, i] for i in range(12))
us = lambda a, b: round(float(np.median((b - a) * 0.01)), 2)   # noqa: E731  (ticks of 10 ns)
info = (ctypes.c_uint64 * 2)()
L.hvws_door_info(None, info)
out = {"reads": n, "busy_chip": busy, "request_in_device_memory": bool(info[0]), "experiment": os.environ.get("HVWS_EXPERIMENT", ""), "host_us_per_call_median": round(float(np.median(wall[n // 10:])) * 1e6, 2),
       "device_us_median": {"request_read": us(t0, t5), "stage": us(t5, t1), "carried_in_frame": us(t1, tw),
                            "walk": us(tw, t2),
                            "walk_parts": {"chase": us(tw, tc), "parse": us(tc, tp), "tail": us(tp, tt),
                                           "to_barrier": us(tt, t2)},
                            "xor_and_stores": us(t2, t3), "xor_parts": {"xor": us(t2, tx), "stores": us(tx, t3)},
                            "records": us(t3, t4)},
       "device_us_total_median": us(t0, t4),
       "release_us_median": round(float(np.median(rel * 0.01)), 2)}   # the previous request's fence + barrier
print(json.dumps(out))
L.hvws_wsp_free(h)
