#!/bin/bash
# round 4: k_build lean form without the records-first branch (6: C=3, no
# VGPR spills, 7 waves per SIMD) against 0 (64 x 4) and 5 (64 x 4 lean, 253
# spilled VGPRs: the staged loads wait on scratch reloads) at c2 / c3 / c4
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4ae}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_BUILD=6 $S pytest_tx_b6_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread -k "not every_geometry and not by_frame_size"
[ -f gpurun_out/.stop ] && exit 1
for rep in 1 2; do
  for cfg in c2 c3 c4; do
    for v in 0 5 6; do
      HVWS_BUILD=$v CONFIG=$cfg $S tx_${cfg}_b${v}_${rep}_$TAG 200 python3 scripts/bench_tx.py
      [ -f gpurun_out/.stop ] && exit 1
    done
  done
done
exit 0
