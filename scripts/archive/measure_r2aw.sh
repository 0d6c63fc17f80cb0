#!/bin/bash
# Round 2: hvws_rx_reads layout probe -- pinned read buffers connection-major
# (reads 160 KiB apart) vs iteration-major (one poll iteration's reads side by side).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2aw}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
MODES=gpu_many,gpu_many_pinned,gpu_many_ring,gpu_pipe,gpu_pipe_ring CONNS=16,256,1024,4096 $S bench_feed_$TAG 400 python3 -u scripts/bench_feed.py
MODES=gpu_many_ring CONNS=4096 $S trace_ring_$TAG 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_ring_$TAG -o t --output-format csv -- python3 -u scripts/bench_feed.py
MODES=gpu_many_pinned CONNS=4096 $S trace_pinned_$TAG 200 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_pinned_$TAG -o t --output-format csv -- python3 -u scripts/bench_feed.py
