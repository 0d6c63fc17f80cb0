#!/bin/bash
# round 4: the resident worker's XOR fused into its stores, chunk by chunk
# (HVWS_DOOR_CXOR, default on) -- door and parity tests (the worker serves
# the reference API by default), then phases and per-call latency with and
# without it
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4am}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S pytest_parity_$TAG 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_validate.py tests/test_gpu_threads.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for rep in 1 2; do
  for x in 1 0; do
    HVWS_DOOR_CXOR=$x $S door_phases_x${x}_${rep}_$TAG 120 python3 scripts/probe/door_phases.py 2000
    [ -f gpurun_out/.stop ] && exit 1
    HVWS_DOOR_CXOR=$x $S dropin_x${x}_${rep}_$TAG 200 python3 scripts/bench_dropin.py 2000
    [ -f gpurun_out/.stop ] && exit 1
  done
done
exit 0
