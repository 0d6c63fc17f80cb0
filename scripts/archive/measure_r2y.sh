#!/bin/bash
# Round 2: k_build_small with a pure-payload fast path and single aligned loads.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2y}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S txtest_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
for s in 0 1; do
  HVWS_BUILD_SMALL=$s CONFIG=c2 $S benchtx_${TAG}_c2_s$s 300 python3 scripts/bench_tx.py
done
