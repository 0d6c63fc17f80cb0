#!/bin/bash
# r6j: is the worker's per-read device time cold-path time?  The instruction-
# cache probe (a 16 KiB straight-line block: first run, again, after 50 us of
# idle polling), and the worker's phase stamps with each request served twice
# (door_twice=1: stamps of the second pass) against once.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S lat_r6j 60 scripts/probe/lat_probe
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=feed_times=1 $S dph_once_r6j 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=feed_times=1,door_twice=1 $S dph_twice_r6j 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=door_twice=1 $S pytest_twice_r6j 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
exit 0
