#!/bin/bash
# Round 2: feeder with spin hand-offs; inline small runs; per-phase times at 4096.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2at}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_feed_$TAG 400 python -u -m pytest tests/test_gpu_feed_many.py -x -q --timeout 120 --timeout-method thread
MODES=gpu_many,gpu_pipe,gpu_pipe_inline,cpu_ref CONNS=1,16,64,256,1024,4096 $S bench_feed_$TAG 400 python3 -u scripts/bench_feed.py
MODES=gpu_pipe CONNS=4096 HVWS_FEED_TIMES=1 $S bench_feed_t4096_$TAG 200 python3 -u scripts/bench_feed.py
MODES=gpu_many CONNS=4096 HVWS_FEED_TIMES=1 $S bench_feed_m4096_$TAG 200 python3 -u scripts/bench_feed.py
