#!/bin/bash
# Round 2: k_small phase clock, host vs device output (probe build).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2am}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
HVWS_SMALL_PROBE=1 HVWS_SMALL_ZC=0 $S feedprobe_${TAG}_host 120 python3 scripts/trace_feed.py
HVWS_SMALL_PROBE=1 HVWS_SMALL_ZC=0 HVWS_PROBE_DEVOUT=1 $S feedprobe_${TAG}_dev 120 python3 scripts/trace_feed.py
