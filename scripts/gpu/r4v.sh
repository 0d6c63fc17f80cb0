#!/bin/bash
# round 4: k_build one-wave 4 KiB tiles as the default (0) against its lean-LDS
# form (5: 16 records, 256 B span slack, 8 waves per SIMD) and the round-3
# geometry (1); rx layout through k_build ($HVWS_BUILD_ID=0) against
# k_build_id; transmit tests for 0 and 5
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4v}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
for v in 0 5; do
  HVWS_BUILD=$v $S pytest_tx_b${v}_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
  [ -f gpurun_out/.stop ] && exit 1
done
for cfg in c2 c3 c4; do
  for v in 0 5 1; do
    HVWS_BUILD=$v CONFIG=$cfg $S tx_${cfg}_b${v}_$TAG 200 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
  for v in 0 5; do
    HVWS_BUILD_ID=0 HVWS_BUILD=$v CONFIG=$cfg $S tx_${cfg}_noid_b${v}_$TAG 200 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
exit 0
