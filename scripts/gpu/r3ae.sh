#!/bin/bash
# round 3 final tree: GPU suite, smoke, default bench, the default bench under
# rocprofv3 (exit with the drop-in thread context released), and the N=2
# rehearsal on one card with every leg on; stops at the first crash
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3ae}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 300 python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S trace_${TAG}_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
HVWS_BENCH_WATCHDOG=60 HVWS_BENCH_DEVICE=0 $S rehearsal2_$TAG 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2
