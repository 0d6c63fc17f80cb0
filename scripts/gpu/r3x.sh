#!/bin/bash
# round 3: default bench alone with a stack watchdog (a hang in r3v), then the
# rest of the closing pass if it finishes
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3x}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
HVWS_BENCH_WATCHDOG=45 $S bench_$TAG 150 python3 -u bench.py
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
$S trace_${TAG}_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
B4="python3 bench.py --config c4 --segments 1 --steps 30 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
$S c4s1_$TAG 200 $B4
$S pmcF_c4s1_$TAG 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF_c4s1_$TAG -o p -- $B4
$S pmcW_c4s1_$TAG 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW_c4s1_$TAG -o p -- $B4
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
HVWS_BENCH_DEVICE=0 $S rehearsal2_$TAG 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2
