#!/bin/bash
# CU-masked discovery stream experiment: c4 (1024), c2, c3 pipelined.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
for k in 0 16 32 64; do
  HVWS_SCAN_CUS=$k $S cu${k}_c4 200 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
  HVWS_SCAN_CUS=$k $S cu${k}_c2 200 python bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx
  HVWS_SCAN_CUS=$k $S cu${k}_c3 200 python bench.py --cpu-seconds 0 --host-gib 0 --no-tx --steps 4
done
