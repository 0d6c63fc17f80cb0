#!/bin/bash
# Round 2: concurrent loop threads, each with its own feeder.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bt}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_threads_$TAG 400 python -u -m pytest tests/test_gpu_threads.py -x -v --timeout 200 --timeout-method thread
