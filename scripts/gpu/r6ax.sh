#!/bin/bash
# r6ax: the cut frame's record emitted in the walk's pass by the lane that parsed it; its carry from that lane's fields (no second parse)
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6ax 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
OLD=build/ab/libhvws_head.so
i=0
for v in old new new old old new; do
  i=$((i+1))
  if [ $v = old ]; then HVWS_LIB=$OLD $S dropin_${v}${i}_r6ax 200 python3 scripts/bench_dropin.py
  else $S dropin_${v}${i}_r6ax 200 python3 scripts/bench_dropin.py; fi
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_EXPERIMENT=feed_times=1 $S dph_new_r6ax 200 python3 scripts/probe/door_phases.py 4000
exit 0
