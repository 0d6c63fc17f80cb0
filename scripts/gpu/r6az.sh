#!/bin/bash
# r6az: the door tests with the carried-payload alignment sweep
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6az 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
exit 0
