#!/bin/bash
# Round 2: per-read latency after caching the pinned buffers' device addresses
# and rate-limiting the stream queries of the completion poll.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bf}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_small_$TAG 400 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_rx_reads.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "feed or reads or execute or parser or quirk"
for rep in 1 2 3; do
  $S perread_${TAG}_$rep 120 python3 scripts/trace_feed.py
done
MODES=gpu_many,gpu_pipe_ring,cpu_ref CONNS=1,16,64 $S benchfeed_$TAG 300 python3 -u scripts/bench_feed.py
READS=200 $S trace_perread_$TAG 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d gpurun_out/trace_perread_$TAG -o t --output-format csv -- python3 scripts/trace_feed.py
