#!/bin/bash
# round 4: k_build's grid-stride form (the next tile's frame range and span
# load while the current tile builds) -- transmit tests with each loop
# variant, then c2 and c3 shapes alternated against the default
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4l}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
for v in 5 6; do
  HVWS_BUILD=$v $S pytest_tx_b${v}_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
  [ -f gpurun_out/.stop ] && exit 1
done
for i in 1 2; do
  for v in 0 5 6; do
    HVWS_BUILD=$v CONFIG=c2 $S tx_c2_b${v}_${i}_$TAG 120 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
for v in 0 5 6; do
  HVWS_BUILD=$v CONFIG=c3 $S tx_c3_b${v}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
