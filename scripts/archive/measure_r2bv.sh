#!/bin/bash
# Round 2, final tree: kernel trace of the pinned pipelined event loop
# (1024 and 4096 connections) for the k_small dispatch durations.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bv}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for c in 1024 4096; do
  MODES=gpu_pipe_ring CONNS=$c $S trace_feed${c}_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_feed${c}_$TAG -o t --output-format csv -- python3 -u scripts/bench_feed.py
done
