#!/bin/bash
# Round 2: event-loop threads (scripts/feed_mt.cpp) with the feeder (50 us hand-off spin) and
# pinned in-place reads, beside the synchronous batched call and the reference.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ay}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
MODES="gpu gpupipe gpupin gpupinpipe ref" CONNS="1024" THREADS="1 4 8" $S feed_mt_$TAG 600 bash scripts/feed_mt.sh
MODES=gpu_many,gpu_pipe,gpu_many_ring,gpu_pipe_ring CONNS=16,64,1024,4096 $S bench_feed_$TAG 300 python3 -u scripts/bench_feed.py
