"""Does hvws_dev_free return a c3-sized rx buffer after each kind of
operation?  (Before the empty-launch fix, hipFree after hvws_digest or
hvws_step left the 68.7 GB allocated.)"""
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
    rx.free()   # hvws_dev_free
    print(name, "freed", free_gb(), flush=True)
    if free_gb() < 150:
        print("stopping: memory held", flush=True)
        break
dp.free()
eng.close()
print("closed", free_gb(), flush=True)
