#!/bin/bash
# round 4: the resident worker with the record-major XOR in LDS and no HIP
# call on its fast path (door tests, ASan, phases on an idle and a busy chip,
# per-call latency); transmit with k_build at 64 VGPRs; then the whole GPU
# suite with the worker on
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4g}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
ASAN_OPTIONS=detect_leaks=0 $S asan_door_$TAG 180 build/asan/asan_driver door
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
DOOR_PHASES_BUSY=1 $S door_phases_busy_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  CONFIG=c2 $S tx_c2_${i}_$TAG 120 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_DOOR=1 $S pytest_gpu_door_on_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
exit 0
