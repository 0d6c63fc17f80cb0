#!/bin/bash
# round 4: k_build's boundary tiles with one 32-byte tile-relative record per
# frame (variant 0) against the 64-bit per-field arrays (variant 5): transmit
# and validation tests, c2 and c3 shapes alternated, then k_build's HBM
# traffic at the c2 shape (separate FETCH_SIZE / WRITE_SIZE passes)
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4m}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_tx_$TAG 400 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  for v in 0 5; do
    HVWS_BUILD=$v CONFIG=c2 $S tx_c2_b${v}_${i}_$TAG 120 python3 scripts/bench_tx.py
    [ -f gpurun_out/.stop ] && exit 1
  done
done
for v in 0 5; do
  HVWS_BUILD=$v CONFIG=c3 $S tx_c3_b${v}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
CONFIG=c2 REPS=2 $S pmcF_tx_c2_$TAG 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
[ -f gpurun_out/.stop ] && exit 1
CONFIG=c2 REPS=2 $S pmcW_tx_c2_$TAG 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW_tx_c2_$TAG -o run --output-format csv -- python3 scripts/bench_tx.py
exit 0
