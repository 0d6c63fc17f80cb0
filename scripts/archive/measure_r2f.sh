#!/bin/bash
# Round 2: c2 / c4 pipelined, k_verify pair forced (1) vs adaptive (-1),
# 200 steps, interleaved 3 times (the 40-step runs of r2e differed by 10 %).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2f}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
B="python3 bench.py --steps 200 --warmup 10 --cpu-seconds 0 --host-gib 0 --no-tx"
for rep in 1 2 3; do
  for v in 1 -1; do
    HVWS_WALK_VERIFY=$v $S bench_${TAG}_c2_v${v}_$rep 200 $B --config c2
    HVWS_WALK_VERIFY=$v $S bench_${TAG}_c4_v${v}_$rep 200 $B --config c4 --segments 1024
  done
done
HVWS_WALK_VERIFY=1 $S trace_${TAG}_c2_v1 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2_v1 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
