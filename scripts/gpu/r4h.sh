#!/bin/bash
# round 4: the worker's staging and store phases -- a probe of one
# workgroup's 8 KiB loads and stores by memory kind and form, then the worker
# with nontemporal data loads and/or the data's first chunks loaded in the
# request's round trip (phases and per-call latency, alternated), and the
# door tests with both knobs on
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4h}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S stage_probe_$TAG 60 build/stage_probe
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  for v in "0 0" "1 0" "0 1" "1 1"; do
    set -- $v
    HVWS_DOOR_NT=$1 HVWS_DOOR_PRELOAD=$2 $S door_phases_nt$1_pre$2_${i}_$TAG 120 python3 scripts/probe/door_phases.py 2000
    [ -f gpurun_out/.stop ] && exit 1
    HVWS_DOOR_NT=$1 HVWS_DOOR_PRELOAD=$2 $S dropin_nt$1_pre$2_${i}_$TAG 200 python3 scripts/bench_dropin.py 2000
    [ -f gpurun_out/.stop ] && exit 1
  done
done
HVWS_DOOR_NT=1 HVWS_DOOR_PRELOAD=1 $S pytest_door_knobs_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
exit 0
