#!/bin/bash
# lazy speculative-table check: parity, then c2/c3/c4 lazy vs waiting
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
$S lazy_parity 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 0
grep -q " passed" gpurun_out/lazy_parity.log && ! grep -q "failed" gpurun_out/lazy_parity.log || exit 0
for cfg in c2 c3; do
  $S lz_${cfg}_lazy 300 python bench.py --config $cfg --cpu-seconds 0 --host-gib 0 --no-tx
  $S lz_${cfg}_wait 300 python bench.py --config $cfg --cpu-seconds 0 --host-gib 0 --no-tx --no-lazy
done
$S lz_c4_lazy 300 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
$S lz_c2_trace 300 rocprofv3 --kernel-trace -d gpurun_out/trace_c2lazy -o run --output-format csv -- python bench.py --config c2 --steps 5 --warmup 1 --cpu-seconds 0 --host-gib 0 --no-tx
