#!/bin/bash
# round 3: exit under the profiler -- default bench traced with the resident
# worker off, then on (workers parked and their CU-masked streams destroyed by
# the library's exit handler), then the door/parity subset; stops at the first crash
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3ab}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
HVWS_DOOR=0 $S trace_door0_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_door0_$TAG -o run --output-format csv -- python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S trace_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$TAG -o run --output-format csv -- python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S pytest_doorsub_$TAG 300 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "door or execute or message or decode or build_frame"
