#!/bin/bash
# Round 2: small-batch path (FeedRecvData, hvws_feed_many) with its timing
# events attached to the k_small dispatch vs marker packets
# (HVWS_SMALL_MARKERS=1).  Feed/ABI parity tests, then bench_feed both ways.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2aa}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S feedtest_$TAG 400 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_threads.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "feed or thread or quirk or execute or parser"
for m in 1 0; do
  HVWS_SMALL_MARKERS=$m ITERS=40 $S benchfeed_${TAG}_m$m 300 python3 scripts/bench_feed.py
done
