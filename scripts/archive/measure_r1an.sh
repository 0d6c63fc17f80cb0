#!/bin/bash
# k_build variants: tx parity under each, then c2/c3 tx rates (interleaved)
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
for v in 6 7; do
  HVWS_BUILD=$v $S txtest_$v 300 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_parity.py -k "build" -x -q --timeout 120 --timeout-method thread
done
for cfg in c2 c3; do
  for v in 0 6 7 0 6; do
    HVWS_BUILD=$v $S tx_${cfg}_$v 300 python bench.py --config $cfg --steps 5 --warmup 2 --cpu-seconds 0 --host-gib 0
    mv gpurun_out/tx_${cfg}_$v.log gpurun_out/tx_${cfg}_${v}_$(date +%s%N).log
  done
done
