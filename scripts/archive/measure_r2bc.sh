#!/bin/bash
# Round 2: message contents assembled on the host copy pool before the replay
# (hvws_set_parallel_replay) -- feed / validation / reads tests in both replay
# modes, then the event-loop bench with the parallel replay off and on.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bc}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_replay_$TAG 600 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_validate.py tests/test_gpu_rx_reads.py -x -q --timeout 120 --timeout-method thread
for p in 0 1; do
  HVWS_PAR_REPLAY=$p MODES=gpu_many,gpu_pipe,gpu_many_ring,gpu_pipe_ring CONNS=64,256,1024,4096 $S benchfeed_${TAG}_par$p 300 python3 -u scripts/bench_feed.py
done
for p in 0 1; do
  HVWS_PAR_REPLAY=$p MODES="gpupinpipe ref" CONNS="1024" THREADS="1 4" $S feed_mt_${TAG}_par$p 300 bash scripts/feed_mt.sh
done
