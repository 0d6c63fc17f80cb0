#!/bin/bash
# Round 2: where a single 8 KiB FeedRecvData goes -- HIP runtime API + kernel
# + memory-copy trace of the per-read loop (scripts/trace_feed.py).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2be}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S perread_$TAG 120 python3 scripts/trace_feed.py
READS=200 $S trace_perread_$TAG 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --stats -d gpurun_out/trace_perread_$TAG -o t --output-format csv -- python3 scripts/trace_feed.py
