#!/bin/bash
# Frame sieve, candidate compaction: parity, c4 one-stream bench, trace, PMC.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r1v}
export TMPDIR=/tmp
B="python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx"
$S pytest_parity 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
$S bench_${TAG}_c4_seg1 300 $B --steps 5 --warmup 2
$S trace_${TAG}_c4_seg1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c4_seg1 -o run --output-format csv -- $B --steps 3 --warmup 1
$S pmc_${TAG}_sq1 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d gpurun_out/pmc_${TAG}_sq1 -o run --output-format csv -- $B --steps 1 --warmup 0
