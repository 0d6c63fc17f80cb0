#!/bin/bash
# round 4 (r4ah): the lean k_build form (5) without VGPR spills -- the records-first
# path of its own, one chunk load at a time (66 VGPRs, 7 waves per
# SIMD) -- against 0 at c2 / c3 / c4; every transmit test with the lean form
# forced
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4ah}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_BUILD=5 $S pytest_tx_b5_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread -k "not every_geometry and not by_frame_size"
[ -f gpurun_out/.stop ] && exit 1
for rep in 1 2; do
  for cfg in c2 c3 c4; do
    for v in 0 5; do
      HVWS_BUILD=$v CONFIG=$cfg $S tx_${cfg}_b${v}_${rep}_$TAG 200 python3 scripts/bench_tx.py
      [ -f gpurun_out/.stop ] && exit 1
    done
  done
done
exit 0
