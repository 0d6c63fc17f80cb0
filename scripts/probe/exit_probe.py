"""Probe (diagnostics, not product code): one process that makes one
resident-worker read through the reference API and exits.  Its Python exit
handler copies /proc/self/maps (the C-level finalizers run after it, with the
same libraries mapped), so the frames of a crash at exit can be resolved
against the mapped libraries offline (scripts/probe/symbolize.py).

  python3 scripts/probe/exit_probe.py TAG            # unprofiled
  rocprofv3 --kernel-trace --stats -d gpurun_out/TAG_kt -o kt -- python3 scripts/probe/exit_probe.py TAG
"""
import atexit
import ctypes
import os
import random
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import libhv_amd  # noqa: E402
import streams as S  # noqa: E402
import wsharness as H  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "exit"
out = os.path.join(ROOT, "gpurun_out")
os.makedirs(out, exist_ok=True)

L = libhv_amd.lib()
data = S.rand_stream(random.Random(5), 6, max_len=3000)
assert H.run_messages("gpu", data, [len(data)]) == H.run_messages("oracle", data, [len(data)])
st = (ctypes.c_uint64 * 4)()
L.hvws_door_stats(None, st)
print(f"[exit_probe] door stats {list(st)} (served > 0: the read went to the worker)", flush=True)
assert st[1] > 0 or os.environ.get("HVWS_DOOR") == "0", "the read did not go to the worker"
if os.environ.get("EXIT_PROBE_RELEASE") == "1":
    L.hvws_thread_release()
    print("[exit_probe] thread context released", flush=True)


def _maps():
    shutil.copy("/proc/self/maps", os.path.join(out, f"{tag}_maps.txt"))
    print("[exit_probe] maps written; exiting", flush=True)


if os.environ.get("EXIT_PROBE_MAPS", "1") == "1":
    atexit.register(_maps)
