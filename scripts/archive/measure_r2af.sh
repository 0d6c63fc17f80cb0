#!/bin/bash
# Round 2: k_small staging the segment and its records in LDS: per-read trace, zc on/off,
# then the feed tests.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ag}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for z in 0 1; do
  HVWS_SMALL_ZC=$z $S feedplain_${TAG}_z$z 120 python3 scripts/trace_feed.py
  HVWS_SMALL_ZC=$z $S feedtrace_${TAG}_z$z 200 rocprofv3 --hip-runtime-trace --kernel-trace -d gpurun_out/feedtrace_${TAG}_z$z -o run --output-format csv -- python3 scripts/trace_feed.py
done
$S feedtest_$TAG 500 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_threads.py tests/test_gpu_validate.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "feed or thread or quirk or execute or parser or valid"
