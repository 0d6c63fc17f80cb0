#!/bin/bash
# round 4: lean k_build tiles in two passes -- chunks inside one payload in a
# short form, the chunks holding header bytes or a frame end gathered and
# assembled 64 per pass -- against 0 at c2; c3 / c4 with the default form
# (its code now shares the assembly as a lambda); every transmit test with
# the lean form forced
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4ai}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_BUILD=5 $S pytest_tx_b5_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread -k "not every_geometry and not by_frame_size"
[ -f gpurun_out/.stop ] && exit 1
for rep in 1 2; do
  for v in 0 5; do
    HVWS_BUILD=$v CONFIG=c2 $S tx_c2_b${v}_${rep}_$TAG 200 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
  for cfg in c3 c4; do
    CONFIG=$cfg $S tx_${cfg}_${rep}_$TAG 200 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
exit 0
