#!/bin/bash
# round 4: the worker's record unmask in 32-bit arithmetic with the partial
# chunks on two lanes -- door tests, the whole GPU suite, phases and per-call
# latency twice
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4n}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
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
