#!/bin/bash
# round 3: the worker's serial header walk for a read's first frames --
# door + drop-in parity subset, the phase probe, the drop-in leg; stops at the
# first crash
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3ad}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_doorsub_$TAG 300 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_parity.py tests/test_gpu_feed_many.py -x -q --timeout 120 --timeout-method thread -k "door or execute or message or decode or build_frame or feed"
[ -f gpurun_out/.stop ] && exit 1
grep -q " passed" gpurun_out/pytest_doorsub_$TAG.log && ! grep -q "failed" gpurun_out/pytest_doorsub_$TAG.log || { echo "door tests not green"; exit 1; }
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
