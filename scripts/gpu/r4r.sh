#!/bin/bash
# round 4: k_build's short path for chunks inside one payload (variant 0)
# against the compact records without it (6) and the 64-bit arrays (5):
# transmit tests, c2 shapes alternated twice, c3 once each
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4r}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_BUILD=6 $S pytest_tx_b6_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  for v in 0 6 5; do
    HVWS_BUILD=$v CONFIG=c2 $S tx_c2_b${v}_${i}_$TAG 120 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
for v in 0 6; do
  HVWS_BUILD=$v CONFIG=c3 $S tx_c3_b${v}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
