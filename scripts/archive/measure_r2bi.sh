#!/bin/bash
# Round 2: spread of bench.py's event-loop leg (pipelined feeder vs batched)
# across repeated processes, beside bench_feed's pinned-ring loop.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bi}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for rep in 1 2 3; do
  $S benchel_${TAG}_$rep 200 python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --host-gib 0 --no-tx
  MODES=gpu_many_ring,gpu_pipe_ring CONNS=1024 $S benchfeed_${TAG}_$rep 200 python3 -u scripts/bench_feed.py
done
