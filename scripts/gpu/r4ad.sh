#!/bin/bash
# round 4: robustness of the final tree's resident worker -- the door stress
# probe (worker on/off beside another context's pinned allocations, pipeline
# and frees; 40 rounds, one line each), the door tests and the whole GPU suite
# with released worker streams destroyed ($HVWS_DOOR_POOL=0), the door tests
# with the worker's idle time at 100 us (parks and relaunches all the time)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4ad}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S door_stress_$TAG 300 python3 -u scripts/probe/door_stress.py 40
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_IDLE_US=100 $S pytest_door_idle100_$TAG 300 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_POOL=0 $S pytest_gpu_nopool_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
exit 0
