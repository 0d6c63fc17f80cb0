#!/bin/bash
# r6au: the worker XOR's partial chunks a dword per lane (lanes 0-3 the first chunk, 4-7 the last) instead of four unrolled steps on lanes 0 and 1
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_door_r6au 400 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py tests/test_gpu_parity.py tests/test_gpu_rx_reads.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
OLD=build/ab/libhvws_head.so
i=0
for v in old new new old old new; do
  i=$((i+1))
  if [ $v = old ]; then HVWS_LIB=$OLD $S dropin_${v}${i}_r6au 200 python3 scripts/bench_dropin.py
  else $S dropin_${v}${i}_r6au 200 python3 scripts/bench_dropin.py; fi
  [ -f gpurun_out/.stop ] && exit 1
done
HVWS_EXPERIMENT=feed_times=1 $S dph_new_r6au 200 python3 scripts/probe/door_phases.py 4000
exit 0
