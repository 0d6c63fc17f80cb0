#!/bin/bash
# Round 2: zero-copy reads for large small-path batches (HVWS_ZC_BATCH) and
# a kernel/copy trace of one 4096-connection poll loop.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2au}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for zb in 1048576 67108864; do
  HVWS_ZC_BATCH=$zb MODES=gpu_many,gpu_pipe CONNS=256,1024,4096 $S bench_feed_zb${zb}_$TAG 300 python3 -u scripts/bench_feed.py
done
for zb in 1048576 67108864; do
  HVWS_ZC_BATCH=$zb MODES=gpu_many CONNS=4096 $S trace_zb${zb}_$TAG 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/trace_zb${zb}_$TAG -o t --output-format csv -- python3 -u scripts/bench_feed.py
done
