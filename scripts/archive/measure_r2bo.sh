#!/bin/bash
# Round 2: k_small's record-major XOR taking each record's fields by readlane
# (one LDS round trip per record instead of two) -- small-path tests, then the
# per-read loop with the previous library (build/alt/libhvws_base.so) and the
# new one swapped in turn (same box, interleaved).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bo}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
cp build/alt/libhvws_new.so libhv_amd/libhvws.so
$S pytest_small_$TAG 500 python -u -m pytest tests/test_gpu_feed_many.py tests/test_gpu_rx_reads.py tests/test_gpu_parity.py tests/test_gpu_threads.py tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread -k "feed or reads or execute or parser or quirk or thread or valid or small or density"
for rep in 1 2 3; do
  for v in base new; do
    cp build/alt/libhvws_$v.so libhv_amd/libhvws.so
    $S perread_${TAG}_${v}_$rep 120 python3 scripts/trace_feed.py
  done
done
for v in base new; do
  cp build/alt/libhvws_$v.so libhv_amd/libhvws.so
  MODES=gpu_many,gpu_pipe_ring CONNS=1,16,64,1024 $S benchfeed_${TAG}_$v 300 python3 -u scripts/bench_feed.py
done
cp build/alt/libhvws_new.so libhv_amd/libhvws.so
