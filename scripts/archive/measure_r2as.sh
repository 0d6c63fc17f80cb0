#!/bin/bash
# Round 2: pipelined feeder (hvws_feeder) -- feed tests, then the event-loop
# bench with the pipelined mode beside the synchronous batched one.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2as}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_feed_$TAG 400 python -u -m pytest tests/test_gpu_feed_many.py -x -v --timeout 120 --timeout-method thread
MODES=gpu_many,gpu_pipe,cpu_ref CONNS=1,16,256,1024,4096 HVWS_FEED_TIMES=1 $S bench_feed_$TAG 400 python3 -u scripts/bench_feed.py
