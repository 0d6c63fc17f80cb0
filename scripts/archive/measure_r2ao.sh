#!/bin/bash
# Round 2: k_small staged in LDS (record-major XOR, store-only host pass),
# untimed plain launch, zero-copy for small batches.  Feed/parity tests, the
# per-read loop, bench_feed with zero-copy on and off.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ao}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S feedtest_$TAG 500 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_threads.py tests/test_gpu_validate.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "feed or thread or quirk or execute or parser or valid"
for z in 1 0; do
  HVWS_SMALL_ZC=$z $S feedplain_${TAG}_z$z 120 python3 scripts/trace_feed.py
  HVWS_SMALL_ZC=$z ITERS=40 $S benchfeed_${TAG}_z$z 300 python3 scripts/bench_feed.py
done
