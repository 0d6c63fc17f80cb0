#!/bin/bash
# Round 2: c4 one-stream (frame sieve) kernel trace with the round-2 engine,
# and FETCH_SIZE / WRITE_SIZE passes for c2 (k_unmask<512,2,linear>).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2o}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
B="--cpu-seconds 0 --host-gib 0 --no-tx"
$S trace_${TAG}_c4seg1 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c4seg1 -o run --output-format csv -- python3 bench.py --config c4 --segments 1 --steps 20 --warmup 5 $B
$S pmc_fetch_c2_${TAG} 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_c2_$TAG -o run --output-format csv -- python3 bench.py --config c2 --steps 2 --warmup 0 $B
$S pmc_write_c2_${TAG} 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_c2_$TAG -o run --output-format csv -- python3 bench.py --config c2 --steps 2 --warmup 0 $B
