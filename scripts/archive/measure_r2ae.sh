#!/bin/bash
# Round 2: runtime trace of the per-read FeedRecvData loop, zero-copy on/off.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ae}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for z in 0 1; do
  HVWS_SMALL_ZC=$z $S feedplain_${TAG}_z$z 120 python3 scripts/trace_feed.py
  HVWS_SMALL_ZC=$z $S feedtrace_${TAG}_z$z 200 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d gpurun_out/feedtrace_${TAG}_z$z -o run --output-format csv -- python3 scripts/trace_feed.py
done
