#!/bin/bash
# Round 2, re-created container: validate HEAD on a fresh box -- GPU suite,
# smoke, default bench, then the N=2 replica rehearsal on the one card.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2ar}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 300 python3 bench.py
HVWS_BENCH_DEVICE=0 $S bench2_$TAG 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 5 --warmup 2
