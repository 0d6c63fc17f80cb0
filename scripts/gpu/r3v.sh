#!/bin/bash
# round 3 closing-style pass: GPU suite, smoke, default bench, kernel trace of
# the default bench, c4 one-stream step traffic (two PMC passes), the drop-in
# latency leg, and the N=2 rehearsal on one card with every leg on
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3v}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
$S bench_$TAG 400 python3 bench.py
$S trace_${TAG}_c3 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
B4="python3 bench.py --config c4 --segments 1 --steps 30 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
$S c4s1_$TAG 200 $B4
$S pmcF_c4s1_$TAG 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF_c4s1_$TAG -o p -- $B4
$S pmcW_c4s1_$TAG 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW_c4s1_$TAG -o p -- $B4
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
HVWS_BENCH_DEVICE=0 $S rehearsal2_$TAG 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2
