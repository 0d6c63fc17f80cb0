#!/bin/bash
# Round 2: software prefetch of the next connections' read bytes during the
# replay ($HVWS_REPLAY_PREFETCH bytes; 0 = off), interleaved A/B/C twice.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bd}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_feed_$TAG 300 python -u -m pytest tests/test_gpu_feed_many.py -x -q --timeout 120 --timeout-method thread
for rep in 1 2; do
  for pf in 0 16384 65536; do
    HVWS_REPLAY_PREFETCH=$pf MODES=gpu_many_ring,gpu_pipe_ring,gpu_pipe CONNS=256,1024,4096 $S benchfeed_${TAG}_pf${pf}_$rep 300 python3 -u scripts/bench_feed.py
  done
done
