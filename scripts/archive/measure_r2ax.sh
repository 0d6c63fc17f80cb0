#!/bin/bash
# Round 2: event-loop threads (scripts/feed_mt.cpp) with the feeder (200 us hand-off spin) and
# pinned in-place reads, beside the synchronous batched call and the reference.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ax}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
MODES="gpu gpupipe gpupin gpupinpipe ref" CONNS="256 1024" THREADS="1 2 4 8" $S feed_mt_$TAG 600 bash scripts/feed_mt.sh
