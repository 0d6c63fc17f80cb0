#!/bin/bash
# Round 2: k_small completion words polled by the host instead of a stream
# sync ($HVWS_SMALL_POLL): small-path parity tests, then per-read latency and
# the event-loop bench with polling off and on.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ba}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_small_$TAG 600 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_rx_reads.py tests/test_gpu_threads.py tests/test_gpu_validate.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "feed or thread or quirk or execute or parser or valid or reads or batch"
for p in 0 1 0 1; do
  HVWS_SMALL_POLL=$p $S perread_${TAG}_p$p 120 python3 scripts/trace_feed.py
done
for p in 0 1; do
  HVWS_SMALL_POLL=$p MODES=gpu_many,gpu_pipe_ring,gpu_many_ring CONNS=1,16,64,1024 $S benchfeed_${TAG}_p$p 300 python3 -u scripts/bench_feed.py
done
