#!/bin/bash
# Round 2: feed tests with the feeder's inline path added.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bl}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_feed_$TAG 400 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_rx_reads.py -x -q --timeout 120 --timeout-method thread
