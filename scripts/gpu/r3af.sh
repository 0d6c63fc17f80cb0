#!/bin/bash
# round 3: c4 one-stream step traffic with the windowed sieve -- two separate
# PMC passes (FETCH_SIZE, WRITE_SIZE) over the same 30-step bench command
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3af}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/.stop
B4="python3 bench.py --config c4 --segments 1 --steps 30 --warmup 3 --cpu-seconds 0 --host-gib 0 --no-tx --feed-conns 0 --dropin-reads 0"
$S pmcF_c4s1_$TAG 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF_c4s1_$TAG -o p -- $B4
[ -f gpurun_out/.stop ] && exit 1
$S pmcW_c4s1_$TAG 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW_c4s1_$TAG -o p -- $B4
[ -f gpurun_out/.stop ] && exit 1
HVWS_SIEVE_HOPS=0 $S pmcF_c4s1_full_$TAG 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF_c4s1_full_$TAG -o p -- $B4
[ -f gpurun_out/.stop ] && exit 1
HVWS_SIEVE_HOPS=0 $S pmcW_c4s1_full_$TAG 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW_c4s1_full_$TAG -o p -- $B4
