#!/bin/bash
# Unmask in pieces (pipelined steps): c4 (1024), c2, c3 for 1/2/4/8 pieces.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
for p in 1 2 4 8; do
  HVWS_UNMASK_PIECES=$p $S pieces${p}_c4 200 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
  HVWS_UNMASK_PIECES=$p $S pieces${p}_c2 200 python bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx
  HVWS_UNMASK_PIECES=$p $S pieces${p}_c3 200 python bench.py --cpu-seconds 0 --host-gib 0 --no-tx --steps 6
done
