#!/usr/bin/env python3
"""The literal drop-in's per-call latency alone (bench.py's drop_in leg, which
runs this script as a child process):
FeedRecvData per 8 KiB read and a masked 125-byte websocket_build_frame, with
the resident worker on and off, and the reference on one core."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import libhv_amd  # noqa: E402

reads = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
device = int(sys.argv[2]) if len(sys.argv) > 2 else 0
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 77
with libhv_amd.Engine(device) as eng:
    print(json.dumps(bench.dropin_leg(eng, device, seed, reads, passes=5)), flush=True)
