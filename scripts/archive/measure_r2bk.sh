#!/bin/bash
# Round 2, end of the last session: event-loop threads (feed_mt) and the
# single-loop sweep (bench_feed) on the final tree.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bk}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
MODES="gpu gpupinpipe ref" CONNS="1024" THREADS="1 2 4 8" $S feed_mt_$TAG 400 bash scripts/feed_mt.sh
MODES=gpu_many,gpu_pipe,gpu_many_ring,gpu_pipe_ring,cpu_ref CONNS=1,16,64,256,1024,4096 $S benchfeed_$TAG 300 python3 -u scripts/bench_feed.py
