#!/bin/bash
# round 4: the worker's chunk-major unmask ($HVWS_DOOR_CHUNK=1) -- door tests
# and the reference-API suites with it on, then phases and per-call latency
# alternated with the record-major default
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4ab}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
HVWS_DOOR_CHUNK=1 $S pytest_door_chunk_$TAG 300 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_parity.py tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  for c in 0 1; do
    HVWS_DOOR_CHUNK=$c $S door_phases_c${c}_${i}_$TAG 120 python3 scripts/probe/door_phases.py 2000
    [ -f gpurun_out/.stop ] && exit 1
    HVWS_DOOR_CHUNK=$c $S dropin_c${c}_${i}_$TAG 200 python3 scripts/bench_dropin.py 2000
    [ -f gpurun_out/.stop ] && exit 1
  done
done
exit 0
