#!/bin/bash
# Round 2: the geometries the serial sweep ranked first at c4 (512x1 XCD,
# 128x2 XCD), pipelined, against 512x2 linear; c2 too.  Interleaved twice.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2t}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx"
for rep in 1 2; do
  for v in 11 2 1; do
    HVWS_UNMASK=$v $S bench_${TAG}_c4_u${v}_$rep 200 $B --steps 100 --warmup 10 --config c4 --segments 1024
    HVWS_UNMASK=$v $S bench_${TAG}_c2_u${v}_$rep 200 $B --steps 200 --warmup 10 --config c2
  done
done
