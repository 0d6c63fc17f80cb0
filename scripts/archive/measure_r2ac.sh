#!/bin/bash
# Round 2: where a feed_many poll iteration's host time goes (HVWS_FEED_TIMES).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ac}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for n in 256 4096; do
  HVWS_FEED_TIMES=1 CONNS=$n MODES=gpu_many ITERS=40 $S feedtimes_${TAG}_$n 200 python3 scripts/bench_feed.py
done
