#!/usr/bin/env python3
"""Diagnostics (not product code): run a Python script with a watchdog that,
every PERIOD seconds the script is still running, prints every thread's
Python stack and native stack (build/libstackdump.so) to stderr -- for a
library build that has no hvws_debug_* calls of its own (the round-3 tree
in which the bench hung).
  scripts/probe/watchdog_run.py PERIOD script.py [args...]"""
import ctypes
import faulthandler
import os
import runpy
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    period = float(sys.argv[1])
    target = os.path.abspath(sys.argv[2])
    sys.argv = [target] + sys.argv[3:]
    sd = ctypes.CDLL(os.path.join(ROOT, "build", "libstackdump.so"))

    def watch():
        n = 0
        while True:
            time.sleep(period)
            n += 1
            print(f"[watchdog] still running after {n * period:.0f} s", file=sys.stderr, flush=True)
            faulthandler.dump_traceback(all_threads=True)
            print(f"[watchdog] native stacks: {sd.sd_backtraces(2)} threads answered", file=sys.stderr, flush=True)

    threading.Thread(target=watch, daemon=True).start()
    sys.path.insert(0, os.path.dirname(target))
    os.chdir(os.path.dirname(target))
    runpy.run_path(target, run_name="__main__")


if __name__ == "__main__":
    main()
