#!/bin/bash
# round 4: the worker's carried-in payload without scalar_frame's state
# dispatch, the walk's carried fields by s_readlane -- door tests, the whole
# GPU suite, phases and per-call latency twice
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4s}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  $S door_phases_${i}_$TAG 120 python3 scripts/probe/door_phases.py 2000
  [ -f gpurun_out/.stop ] && exit 1
  $S dropin_${i}_$TAG 200 python3 scripts/bench_dropin.py 2000
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
