#!/bin/bash
# round 4: the worker stages by LDS-DMA (no register arrays) and reads LDS
# records with ds loads; door tests (default and with preload), then phases
# and per-call latency with and without the preload, alternated
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4i}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_PRELOAD=1 $S pytest_door_pre_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  for p in 0 1; do
    HVWS_DOOR_PRELOAD=$p $S door_phases_pre${p}_${i}_$TAG 120 python3 scripts/probe/door_phases.py 2000
    [ -f gpurun_out/.stop ] && exit 1
    HVWS_DOOR_PRELOAD=$p $S dropin_pre${p}_${i}_$TAG 200 python3 scripts/bench_dropin.py 2000
    [ -f gpurun_out/.stop ] && exit 1
  done
done
exit 0
