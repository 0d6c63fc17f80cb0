#!/bin/bash
# Round 2: in-kernel phase clock of k_small (temporary probe build).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ah}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
for z in 0 1; do
  HVWS_SMALL_PROBE=1 HVWS_SMALL_ZC=$z $S feedprobe_${TAG}_z$z 120 python3 scripts/trace_feed.py
done
