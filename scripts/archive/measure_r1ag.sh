#!/bin/bash
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
$S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
$S bench_default 400 python bench.py
$S trace_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_ag_c4 -o run --output-format csv -- python bench.py --config c4 --segments 1024 --steps 4 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
