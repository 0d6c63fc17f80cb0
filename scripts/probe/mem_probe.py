"""Which operation on a c3-sized rx buffer keeps hipFree from returning its
memory?  For each operation: allocate, build the batch, run it, free with
hipFree directly (its return code printed) and read hipMemGetInfo."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import libhv_amd  # noqa: E402
from libhv_amd import synth  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = ctypes.c_char_p
N = 68734156864 + 64


def free_gb():
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t))
    return round(f.value / 1e9, 2)


eng = libhv_amd.Engine(0)
plan = synth.config_plan("c3", seed=1000).split(4096)
dp = libhv_amd.DevicePlan(eng, plan)
print("start", free_gb(), flush=True)
ops = {
    "synth": lambda rx: None,
    "digest": lambda rx: eng.digest(rx, plan.total),
    "verify": lambda rx: eng.synth(rx, plan.total, plan.seed, dp, 1),
    "scan": lambda rx: eng.scan(rx, plan.total, plan.segments),
    "step": lambda rx: eng.step(rx, plan.total, plan.segments),
    "step_resident": lambda rx: eng.step_resident(rx, plan.total, plan.segments),
}
for name, op in ops.items():
    rx = eng.alloc(N)
    eng.synth(rx, plan.total, plan.seed, dp, 0)
    op(rx)
    eng.sync()
    hip.hipDeviceSynchronize()
    rc = hip.hipFree(ctypes.c_void_p(rx.ptr))
    rx.ptr = None
    print(name, "hipFree", rc, hip.hipGetErrorString(rc).decode(), free_gb(), flush=True)
    if free_gb() < 150:
        print("stopping: memory held", flush=True)
        break
dp.free()
eng.close()
print("closed", free_gb(), flush=True)
