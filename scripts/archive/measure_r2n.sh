#!/bin/bash
# Round 2: c4 (1024 segments, SLACK) unmask pieces with the 512x2 linear
# geometry: HVWS_UNMASK_PIECES 1/2/4/8, interleaved twice.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2n}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx --steps 100 --warmup 10 --config c4 --segments 1024"
for rep in 1 2; do
  for p in 1 2 4 8; do
    HVWS_UNMASK_PIECES=$p $S bench_${TAG}_c4_p${p}_$rep 200 $B
  done
done
# two ranks on one card (the driver's N>1 path, rehearsed): torch.distributed.run, gloo barrier
HVWS_BENCH_DEVICE=0 $S bench_${TAG}_2ranks 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 2 --host-gib 1
