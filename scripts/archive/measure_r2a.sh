#!/bin/bash
# Round-2 profile pass: default bench under a kernel trace, and FETCH_SIZE /
# WRITE_SIZE in separate --pmc passes at c3 and c2 (profiles/traffic.json).
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2a}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S trace_${TAG}_c3 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
$S pmc_fetch_${TAG} 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S pmc_write_${TAG} 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S pmc_fetch_c2_${TAG} 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_c2_$TAG -o run --output-format csv -- python3 bench.py --config c2 --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S pmc_write_c2_${TAG} 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_c2_$TAG -o run --output-format csv -- python3 bench.py --config c2 --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
