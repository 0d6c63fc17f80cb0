#!/bin/bash
# Round 2: N=2 rehearsal of the replica bench on the one-GPU box (both ranks
# on device 0, gloo for the barrier/timing), then N=1 default for comparison.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2aq}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
HVWS_BENCH_DEVICE=0 $S bench2_$TAG 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 5 --warmup 2
