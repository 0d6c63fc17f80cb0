#!/bin/bash
# round 4: where the resident worker's header-walk phase goes (stamps inside door_walk)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4e}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
