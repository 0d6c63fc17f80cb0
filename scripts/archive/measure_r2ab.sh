#!/bin/bash
# Round 2: host copy pool for the batched drop-in.  Feed/thread tests, then
# bench_feed with the pool (default 8 threads) and serial (HVWS_COPY_THREADS=1).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ab}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S feedtest_$TAG 400 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_threads.py -x -q --timeout 120 --timeout-method thread
for t in 8 1; do
  HVWS_COPY_THREADS=$t ITERS=40 $S benchfeed_${TAG}_t$t 300 python3 scripts/bench_feed.py
done
