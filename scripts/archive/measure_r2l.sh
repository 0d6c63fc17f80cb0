#!/bin/bash
# Round 2: unmask geometry per batch size in the real (pipelined) steps.
# HVWS_UNMASK 0 (256x4 xcd, default), 5 (256x2 xcd), 11 (512x2 linear) at
# c2, c4 (1024 segments) and c3, interleaved twice.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2l}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx"
for rep in 1 2; do
  for v in 0 5 11; do
    HVWS_UNMASK=$v $S bench_${TAG}_c2_u${v}_$rep 200 $B --steps 200 --warmup 10 --config c2
    HVWS_UNMASK=$v $S bench_${TAG}_c4_u${v}_$rep 200 $B --steps 100 --warmup 10 --config c4 --segments 1024
    HVWS_UNMASK=$v $S bench_${TAG}_c3_u${v}_$rep 300 $B --steps 20 --warmup 3
  done
done
