#!/bin/bash
# round 4: the transmit tile index and spans fused into three launches (fill,
# one pass over the frames, fixup) instead of six -- transmit tests (every
# geometry, spans on and off), c2 / c3 / c4 twice, then the whole GPU suite
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4ap}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for rep in 1 2; do
  for cfg in c2 c3 c4; do
    CONFIG=$cfg $S tx_${cfg}_${rep}_$TAG 200 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 300 python3 scripts/smoke_run.py
[ -f gpurun_out/.stop ] && exit 1
$S bench_$TAG 400 python3 bench.py
exit 0
