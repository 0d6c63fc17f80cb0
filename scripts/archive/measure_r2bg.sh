#!/bin/bash
# Round 2: the small path skips its leading stream sync after a call that saw
# all its completion words; per-read latency with the words polled vs a
# stream sync at the end (HVWS_SMALL_POLL=1/0), interleaved.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bg}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_small_$TAG 500 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_rx_reads.py tests/test_gpu_parity.py tests/test_gpu_threads.py tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread -k "feed or reads or execute or parser or quirk or thread or valid"
for rep in 1 2 3; do
  for p in 0 1; do
    HVWS_SMALL_POLL=$p $S perread_${TAG}_p${p}_$rep 120 python3 scripts/trace_feed.py
  done
done
for p in 0 1; do
  HVWS_SMALL_POLL=$p MODES=gpu_many,gpu_pipe_ring,gpu_many_ring,cpu_ref CONNS=1,16,64,1024 $S benchfeed_${TAG}_p$p 300 python3 -u scripts/bench_feed.py
done
