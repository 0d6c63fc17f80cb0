#!/bin/bash
# r6o: r6n with the writeback waited for before `done` (the compiler had dropped the wait):
# writeback instead of one per wave): door / feed / parity tests, phase stamps,
# drop-in latency against HEAD's worker (build/ab/libhvws_head.so), interleaved.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6o 400 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=feed_times=1 $S dph_new_r6o 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_LIB=build/ab/libhvws_head.so HVWS_EXPERIMENT=feed_times=1 $S dph_old_r6o 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2 3; do
  $S dropin_new${i}_r6o 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_LIB=build/ab/libhvws_head.so $S dropin_old${i}_r6o 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
