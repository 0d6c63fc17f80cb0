#!/bin/bash
# round 4: k_build's span staged by LDS-DMA in one-wave tiles (6: lean,
# 7: 64 records) against 0 (64 x 4) and 5 (64 x 4 lean): transmit tests, then
# c2 / c3 / c4 shapes alternated
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4ac}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
for v in 6 7; do
  HVWS_BUILD=$v $S pytest_tx_b${v}_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread -k "not every_geometry and not by_frame_size"
  [ -f gpurun_out/.stop ] && exit 1
done
for i in 1 2; do
  for cfg in c2 c3 c4; do
    for v in 0 5 6 7; do
      HVWS_BUILD=$v CONFIG=$cfg $S tx_${cfg}_b${v}_${i}_$TAG 200 python3 scripts/bench_tx.py
      [ -f gpurun_out/.stop ] && exit 1
    done
  done
done
exit 0
