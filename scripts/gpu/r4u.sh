#!/bin/bash
# round 4: k_build with one-wave workgroups (variants 6: 2 KiB tiles, 7: 4 KiB)
# against the 256-thread default at c3 and c4 shapes, and c2 once more
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4u}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
for v in 0 6 7; do
  HVWS_BUILD=$v CONFIG=c3 $S tx_c3_b${v}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
for v in 0 6 7; do
  HVWS_BUILD=$v CONFIG=c4 $S tx_c4_b${v}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
for v in 0 6 7; do
  HVWS_BUILD=$v CONFIG=c2 $S tx_c2_b${v}_$TAG 120 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
