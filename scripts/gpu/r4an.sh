#!/bin/bash
# round 4: k_build lean8 (6: 8 records, 64 B span slack -> 4992 B of LDS and
# 64 VGPRs, 8 tiles per SIMD; the lane id recomputed in the staged block so
# nothing spills there) against lean (5, 7 per SIMD) at c2
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4an}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_BUILD=6 $S pytest_tx_b6_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread -k "not every_geometry and not by_frame_size"
[ -f gpurun_out/.stop ] && exit 1
for rep in 1 2 3; do
  for v in 5 6; do
    HVWS_BUILD=$v CONFIG=c2 $S tx_c2_b${v}_${rep}_$TAG 200 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
exit 0
