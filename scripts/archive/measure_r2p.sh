#!/bin/bash
# Round 2: device-wide scan in 256-thread workgroups (the sieve's scans beside
# a pipelined unmask).  GPU suite, c4 one stream bench + trace, c4 1024 seg.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2p}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx"
$S bench_${TAG}_c4seg1 300 $B --config c4 --segments 1 --steps 40 --warmup 5
$S bench_${TAG}_c4seg1_serial 300 $B --config c4 --segments 1 --steps 40 --warmup 5 --serial
$S trace_${TAG}_c4seg1 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c4seg1 -o run --output-format csv -- python3 bench.py --config c4 --segments 1 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
