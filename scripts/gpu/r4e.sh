#!/bin/bash
# round 4: the resident worker's faster walk (stamps inside door_walk), per-call
# latency; transmit with the segmented span atomics and its kernel trace
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4e}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 $S tx_c2_$TAG 120 python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 $S trace_tx_c2_$TAG 180 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
