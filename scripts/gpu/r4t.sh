#!/bin/bash
# round 4: k_build with smaller workgroups (64 or 128 threads: less to wait
# for at the staging barrier, more tiles in flight per CU) against the
# 256-thread default -- transmit tests per variant, c2 alternated twice, c3
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4t}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
for v in 0 6 7 8; do
  HVWS_BUILD=$v $S pytest_tx_b${v}_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
  [ -f gpurun_out/.stop ] && exit 1
done
for i in 1 2; do
  for v in 0 6 7 8; do
    HVWS_BUILD=$v CONFIG=c2 $S tx_c2_b${v}_${i}_$TAG 120 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
for v in 0 8; do
  HVWS_BUILD=$v CONFIG=c3 $S tx_c3_b${v}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
