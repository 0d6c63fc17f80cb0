#!/bin/bash
# r6ad: c4 at 4096 segments (mixed frames, SLACK scans) on the final tree, twice.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
for i in 1 2; do
  $S c4_r6ad_$i 240 python3 bench.py --config c4 --steps 40 --warmup 5 --no-tx --feed-conns 0 --dropin-reads 0 --host-gib 0 --cpu-seconds 0
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
