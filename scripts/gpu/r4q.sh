#!/bin/bash
# round 4: the tree after the uniform transmit kernel's removal, with worker
# streams pooled -- door and transmit tests, the whole GPU suite, smoke, the
# default bench twice, the default bench under a kernel trace with released
# worker streams destroyed ($HVWS_DOOR_POOL=0), the worker's phases and
# per-call latency, transmit shapes
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4q}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 300 python3 scripts/smoke_run.py
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  $S bench_${i}_$TAG 400 python3 bench.py
  [ -f gpurun_out/.stop ] && exit 1
done
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 $S tx_c2_$TAG 120 python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
HVWS_DOOR_POOL=0 $S trace_c3_$TAG 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c3_$TAG -o run --output-format csv -- python3 bench.py
exit 0
