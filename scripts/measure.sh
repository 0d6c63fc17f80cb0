#!/bin/bash
# One measurement pass on the GPU box (used with gpurun).  Each step has its
# own time limit; a crash/timeout stops the remaining GPU steps.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1}
export TMPDIR=/tmp
$S bench_$TAG 400 python bench.py --sweep-unmask
$S bench_${TAG}_c3_seg1 300 python bench.py --segments 1 --cpu-seconds 0 --host-gib 0 --steps 5
$S bench_${TAG}_c2 300 python bench.py --config c2 --cpu-seconds 2 --host-gib 1 --sweep-unmask
$S bench_${TAG}_c2_seg1 300 python bench.py --config c2 --segments 1 --cpu-seconds 0 --host-gib 0 --steps 5
$S bench_${TAG}_c4 300 python bench.py --config c4 --segments 1024 --cpu-seconds 2 --host-gib 1
$S prof_${TAG} 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0
$S pmc_fetch_${TAG} 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S pmc_write_${TAG} 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S pmc_fetch_c2_${TAG} 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_c2_$TAG -o run --output-format csv -- python bench.py --config c2 --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
$S pmc_write_c2_${TAG} 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_c2_$TAG -o run --output-format csv -- python bench.py --config c2 --steps 2 --warmup 0 --cpu-seconds 0 --host-gib 0
