#!/bin/bash
# r6x: the door tests with the new pinned-request child test; the door / feed
# tests once more with the request area in pinned host memory (door_vram=0).
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6x 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=door_vram=0 $S pytest_door_pinned_r6x 300 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py -x -q --timeout 120 --timeout-method thread
exit 0
