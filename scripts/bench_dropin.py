#!/usr/bin/env python3
"""The literal drop-in's per-call latency alone (bench.py's drop_in leg):
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
with libhv_amd.Engine(0) as eng:
    print(json.dumps(bench.dropin_leg(eng, 0, 77, reads, passes=5)), flush=True)
