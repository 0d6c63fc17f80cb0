#!/bin/bash
# r6aw: the walk publishes each round's records and waves 1-7 unmask them meanwhile; wave 0 unmasks the cut frame itself
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6aw 400 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py tests/test_gpu_parity.py tests/test_gpu_rx_reads.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
OLD=build/ab/libhvws_head.so
i=0
for v in old new new old old new; do
  i=$((i+1))
  if [ $v = old ]; then HVWS_LIB=$OLD $S dropin_${v}${i}_r6aw 200 python3 scripts/bench_dropin.py
  else $S dropin_${v}${i}_r6aw 200 python3 scripts/bench_dropin.py; fi
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_EXPERIMENT=feed_times=1 $S dph_new_r6aw 200 python3 scripts/probe/door_phases.py 4000
exit 0
