#!/bin/bash
# Round 2: hvws_rx_reads (reads in registered pinned memory, no stage) --
# its parity tests, the feed tests, then the event-loop bench with pinned
# read buffers beside pageable ones.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2av}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_reads_$TAG 500 python -u -m pytest tests/test_gpu_rx_reads.py tests/test_gpu_feed_many.py -x -q --timeout 120 --timeout-method thread
MODES=gpu_many,gpu_pipe,gpu_many_pinned,gpu_pipe_pinned,cpu_ref CONNS=1,16,64,256,1024,4096 $S bench_feed_$TAG 400 python3 -u scripts/bench_feed.py
MODES=gpu_pipe_pinned CONNS=4096 HVWS_FEED_TIMES=1 $S bench_feed_t4096_$TAG 200 python3 -u scripts/bench_feed.py
MODES=gpu_many_pinned CONNS=4096 HVWS_FEED_TIMES=1 $S bench_feed_m4096_$TAG 200 python3 -u scripts/bench_feed.py
