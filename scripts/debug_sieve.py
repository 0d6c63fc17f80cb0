"""Per-step sieve diagnostics for one-segment c4 steps (serial and pipelined)."""
import ctypes
import sys
import time

sys.path.insert(0, ".")
import libhv_amd
from libhv_amd import synth

L = libhv_amd.lib()
eng = libhv_amd.Engine(0)
plan = synth.config_plan("c4", seed=1000).split(1)
dp = libhv_amd.DevicePlan(eng, plan)
rx = eng.alloc(plan.total + 64)
eng.synth(rx, plan.total, plan.seed, dp, 0)
eng.sync()
segs = eng.prepare(plan.segments)
out = (ctypes.c_uint64 * 4)()
for mode in ("serial", "resident", "resident_nosync"):
    f = eng.step if mode == "serial" else eng.step_resident
    for i in range(6):
        t = time.perf_counter()
        f(rx, plan.total, segs)
        if mode != "resident_nosync":
            eng.sync()
            L.hvws_last_sieve(eng.ctx, out)
            print(mode, i, f"{(time.perf_counter() - t) * 1e3:.2f} ms", list(out), flush=True)
    eng.sync()
    L.hvws_last_sieve(eng.ctx, out)
    print(mode, "end", list(out), [f"{a:.2f}/{b:.2f}" for a, b in eng.step_times(6)], flush=True)
