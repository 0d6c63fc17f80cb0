#!/bin/bash
# r6i: fence costs (lat_probe); the worker without its system-scope acquire
# (door_acq=0: system-scope loads of the request instead) -- door tests, then
# drop-in latency and phase stamps against the default, interleaved; the suite.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S lat_r6i 60 scripts/probe/lat_probe
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=door_acq=0 $S pytest_door_noacq_r6i 400 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2 3; do
  $S dropin_def${i}_r6i 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
  HVWS_EXPERIMENT=door_acq=0 $S dropin_noacq${i}_r6i 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_EXPERIMENT=feed_times=1 $S dph_def_r6i 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
HVWS_EXPERIMENT=feed_times=1,door_acq=0 $S dph_noacq_r6i 200 python3 scripts/probe/door_phases.py 4000
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_r6i 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
exit 0
