"""Which scan path each step of a resident uniform batch takes (FUSED auto)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import libhv_amd
from libhv_amd import synth
from tests import wsharness as H

L = libhv_amd.lib()
e = libhv_amd.Engine(0)
print("vmask/mode", L.hvws_set_fused(e.ctx, 2))
for n, size, nseg in ((20000, 1024, 64), (2000, 1024, 13)):
    plan = synth.uniform_plan(n, size, 17).split(nseg)
    host = H.synth_cpu(plan)
    rx = e.to_device(host)
    out = (ctypes.c_uint64 * 2)()
    for i in range(6):
        (e.step if i == 0 else e.step_resident)(rx, plan.total, plan.segments)
        e.sync()
        L.hvws_fused_stats(e.ctx, out)
        print(n, size, nseg, i, "path", L.hvws_last_scan_path(e.ctx), "stats", out[0], out[1], flush=True)
    rx.free()
