#!/bin/bash
# r6k: the worker's read restructured (speculative staging beside the request
# block, branch-free chase with uniform control, the parse on all four waves,
# records copied beside the XOR): door / feed / parity tests first, then the
# phase stamps and the drop-in latency, then the whole suite.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6k 400 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=feed_times=1 $S dph_r6k 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2; do
  $S dropin${i}_r6k 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
done
$S pytest_gpu_r6k 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
exit 0
