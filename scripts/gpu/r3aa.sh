#!/bin/bash
# round 3: exit-time heap corruption after the door/parity subset (r3y) --
# the same subset with glibc's malloc checks and a Python stack on a fatal
# signal, once with the worker on and once off; then the door phase probe.
# Any crash or abort ends the call there (scripts/gpu_step.sh writes .stop).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3aa}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
K="door or execute or message or decode or build_frame"
MALLOC_CHECK_=3 MALLOC_PERTURB_=165 $S pytest_doorsub_on_$TAG 300 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K"
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR=0 MALLOC_CHECK_=3 MALLOC_PERTURB_=165 $S pytest_doorsub_off_$TAG 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K"
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
