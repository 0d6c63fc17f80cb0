#!/bin/bash
# r6m: the worker's read, second form (no atomics in the parse, the carried
# fields from the records, the parse without violation classes when validation
# is off, branch-free partial-chunk XOR): door / feed / parity tests, phase
# stamps, drop-in latency against HEAD's worker, interleaved.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6m 400 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py tests/test_gpu_parity.py tests/test_gpu_validate.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=feed_times=1 $S dph_r6m 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  $S dropin_new${i}_r6m 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_LIB=build/ab/libhvws_head.so $S dropin_old${i}_r6m 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
