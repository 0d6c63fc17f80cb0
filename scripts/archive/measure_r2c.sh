#!/bin/bash
# Round 2: one-launch SPEC scan (k_pscan) -- parity suite, then c2/c3 benches
# with the one-launch scan off and on, then a c2 kernel trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2c}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S parity_$TAG 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx"
for cfg in c2 c3; do
  for p in 0 1; do
    HVWS_PSCAN=$p $S bench_${TAG}_${cfg}_p$p 300 $B --config $cfg
  done
done
HVWS_PSCAN=1 $S trace_${TAG}_c2 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
