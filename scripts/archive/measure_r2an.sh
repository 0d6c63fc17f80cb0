#!/bin/bash
# Round 2: per-read FeedRecvData with and without timing events on k_small
# (HVWS_STEP_EVENTS=0), zero-copy on; plain and under a runtime trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2an}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for ev in 0 2; do
  HVWS_STEP_EVENTS=$ev $S feedplain_${TAG}_e$ev 120 python3 scripts/trace_feed.py
  HVWS_STEP_EVENTS=$ev $S feedtrace_${TAG}_e$ev 200 rocprofv3 --hip-runtime-trace --kernel-trace -d gpurun_out/feedtrace_${TAG}_e$ev -o run --output-format csv -- python3 scripts/trace_feed.py
done
