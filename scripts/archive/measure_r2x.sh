#!/bin/bash
# Round 2: k_build_small (one wave per frame for small-frame transmit batches).
# Transmit parity tests, then bench_tx at c2 and c3 with the small path off (0)
# and on (1), and the default bench's tx leg.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2x}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S txtest_$TAG 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
for s in 0 1; do
  HVWS_BUILD_SMALL=$s CONFIG=c2 $S benchtx_${TAG}_c2_s$s 300 python3 scripts/bench_tx.py
done
CONFIG=c3 REPS=3 $S benchtx_${TAG}_c3 400 python3 scripts/bench_tx.py
