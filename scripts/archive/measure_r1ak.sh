#!/bin/bash
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
$S parity_sieve 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "sieve or single_segment" --timeout 120 --timeout-method thread
$S configs 400 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread
$S ak_c4s 200 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S ak_c3 200 python bench.py --cpu-seconds 0 --host-gib 0 --no-tx --steps 4
$S ak_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_ak_c4s -o run --output-format csv -- python bench.py --config c4 --segments 1 --steps 4 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
