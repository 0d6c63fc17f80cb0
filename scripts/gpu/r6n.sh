#!/bin/bash
# r6n: the worker's release by thread 0 alone after the barrier (one L2
# writeback instead of one per wave): door / feed / parity tests, phase stamps,
# drop-in latency against HEAD's worker (build/ab/libhvws_head.so), interleaved.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6n 400 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py tests/test_gpu_parity.py tests/test_gpu_rx_reads.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=feed_times=1 $S dph_new_r6n 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_LIB=build/ab/libhvws_head.so HVWS_EXPERIMENT=feed_times=1 $S dph_old_r6n 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2 3; do
  $S dropin_new${i}_r6n 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_LIB=build/ab/libhvws_head.so $S dropin_old${i}_r6n 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
