#!/bin/bash
# Round 2: SPEC check folded into the tile scatter (k_tile_scatter_check).
# GPU suite, then c2 pipelined/serial with the fold off (0) and on (1),
# interleaved, c4, c3 default bench (full, with the host and tx legs).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2j}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --steps 200 --warmup 10 --cpu-seconds 0 --host-gib 0 --no-tx"
for rep in 1 2; do
  for f in 0 1; do
    HVWS_FOLD_CHECK=$f $S bench_${TAG}_c2_f${f}_$rep 200 $B --config c2
    HVWS_FOLD_CHECK=$f $S bench_${TAG}_c2_f${f}_serial_$rep 200 $B --config c2 --serial
  done
done
$S bench_${TAG}_c4 200 $B --config c4 --segments 1024
$S bench_${TAG}_c3 400 python3 bench.py
