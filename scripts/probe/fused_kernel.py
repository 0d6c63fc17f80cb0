"""k_fused vs k_unmask kernel time at a BASELINE config (c2 default), serial
steps so each pass is timed alone (hvws_last_times), for $HVWS_FUSED_DBG
probe variants.  Bytes are not checked (the probe variants break them)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import libhv_amd
from libhv_amd import synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
nseg = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
L = libhv_amd.lib()
e = libhv_amd.Engine(0)
plan = synth.config_plan(cfg, seed=1000).split(nseg)
dp = libhv_amd.DevicePlan(e, plan)
rx = e.alloc(plan.total + 64)
e.synth(rx, plan.total, plan.seed, dp, 0)
prep = e.prepare(plan.segments)
for mode in (0, 1):
    L.hvws_set_fused(e.ctx, mode)
    e.step(rx, plan.total, prep)      # exact (learns), or the first fused pass
    ts = []
    for _ in range(20):
        e.step(rx, plan.total, prep)
        ts.append(e.last_times())
    sc = np.mean([t[0] for t in ts[2:]])
    um = np.mean([t[1] for t in ts[2:]])
    print(f"{cfg} fused={mode} dbg={os.environ.get('HVWS_FUSED_DBG', '0')} path={L.hvws_last_scan_path(e.ctx)} "
          f"scan_ms={sc:.3f} unmask_ms={um:.3f}", flush=True)
