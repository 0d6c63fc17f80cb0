#!/bin/bash
# Round 2: flat pointer index instead of std::unordered_set/map for the
# batched drop-in's duplicate cut and the feeder's pending lookup -- feed
# tests, then the event-loop bench with the previous library and the new one
# swapped in turn (same box, interleaved).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bq}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
cp build/alt/libhvws_new.so libhv_amd/libhvws.so
$S pytest_feed_$TAG 400 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_rx_reads.py tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread
for rep in 1 2; do
  for v in base new; do
    cp build/alt/libhvws_$v.so libhv_amd/libhvws.so
    MODES=gpu_many_ring,gpu_pipe_ring,gpu_pipe CONNS=16,256,1024,4096 $S benchfeed_${TAG}_${v}_$rep 300 python3 -u scripts/bench_feed.py
  done
done
cp build/alt/libhvws_new.so libhv_amd/libhvws.so
