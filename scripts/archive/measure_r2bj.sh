#!/bin/bash
# Round 2: default bench with the event-loop leg moved ahead of the
# host-inclusive and transmit legs (twice), plus the N=2 one-card rehearsal.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2bj}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S bench_${TAG}_1 400 python3 bench.py
$S bench_${TAG}_2 400 python3 bench.py
HVWS_BENCH_DEVICE=0 $S bench2_$TAG 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 5 --warmup 2
