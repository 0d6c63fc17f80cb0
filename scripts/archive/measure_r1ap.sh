#!/bin/bash
# tile index without the fill: parity, then c2/c4/c3
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
$S nofill_parity 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 0
grep -q " passed" gpurun_out/nofill_parity.log && ! grep -q "failed" gpurun_out/nofill_parity.log || exit 0
$S nf_c2 300 python bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx
$S nf_c4 300 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
$S nf_c3 300 python bench.py --cpu-seconds 0 --host-gib 0 --no-tx
$S nf_c2_trace 300 rocprofv3 --kernel-trace -d gpurun_out/trace_c2nofill -o run --output-format csv -- python bench.py --config c2 --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
