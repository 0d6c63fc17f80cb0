#!/bin/bash
# r6b: which process ends crash at exit under rocprofv3 -- a bare CU-masked
# stream (no hvws code), destroyed or not, an ordinary stream; then the
# library's one-read process after hvws_thread_release (worker parked, stream
# pooled).  Expected-clean runs first: a crash ends the call.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
P=scripts/probe/cumask_exit
for m in 2 1 3 0; do
  $S cumask_m${m}_plain_r6b 30 $P $m
  [ -f gpurun_out/.stop ] && exit 1
done
for m in 2 1 3 0; do
  $S cumask_m${m}_kt_r6b 60 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_kt_m$m -o kt -- $P $m
  [ -f gpurun_out/.stop ] && exit 1
done
EXIT_PROBE_RELEASE=1 $S exit_rel_kt_r6b 90 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_kt_rel -o kt -- python3 scripts/probe/exit_probe.py rel_r6b
exit 0
