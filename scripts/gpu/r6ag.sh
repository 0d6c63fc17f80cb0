#!/bin/bash
# r6ag: the worker's width -- 4 waves (HEAD, build/ab/libhvws_head.so), 8 waves
# (build/ab/libhvws_t512.so), 12 waves (tree) -- drop-in latency in rotating
# order, three rounds, and the phase stamps of each.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
lib() { case $1 in w4) echo build/ab/libhvws_head.so;; w8) echo build/ab/libhvws_t512.so;; w12) echo libhv_amd/libhvws.so;; esac; }
i=0
for v in w4 w8 w12 w12 w8 w4 w8 w4 w12; do
  i=$((i+1))
  HVWS_LIB=$(lib $v) $S dropin_${v}_${i}_r6ag 200 python3 scripts/bench_dropin.py
  [ -f gpurun_out/.stop ] && exit 1
done
for v in w4 w8 w12; do
  HVWS_LIB=$(lib $v) HVWS_EXPERIMENT=feed_times=1 $S dph_${v}_r6ag 200 python3 scripts/probe/door_phases.py 4000
  [ -f gpurun_out/.stop ] && exit 1
done
$S pytest_door_r6ag 300 python -u -m pytest tests/test_gpu_door.py tests/test_gpu_feed_many.py -x -q --timeout 120 --timeout-method thread
exit 0
