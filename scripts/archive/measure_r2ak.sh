#!/bin/bash
# Round 2: k_small with batched staging loads and a store-only host pass:
# in-kernel phase clock (probe build), then the feed/parity tests.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ak}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for z in 0 1; do
  HVWS_SMALL_PROBE=1 HVWS_SMALL_ZC=$z $S feedprobe_${TAG}_z$z 120 python3 scripts/trace_feed.py
done
$S feedtest_$TAG 500 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_threads.py tests/test_gpu_validate.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "feed or thread or quirk or execute or parser or valid"
