#!/bin/bash
# round 4: k_build_uni with reciprocal divisions; worker streams pooled --
# c2 and c3 shapes twice; door tests first (their stuck-thread helper now
# dumps native stacks and mailboxes; worker streams drain with bounds)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4p}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  CONFIG=c2 $S tx_c2_${i}_$TAG 120 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
CONFIG=c3 $S tx_c3_$TAG 200 python3 scripts/bench_tx.py
exit 0
