#!/bin/bash
# Round 2: pipelined SPEC tail (check + tile kernels) on the unmask stream.
# Parity, then c2/c3 with the tail on the scan stream (HVWS_TAIL=0) and on the
# unmask stream (1), interleaved, and a c2 kernel trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2g}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S parity_$TAG 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --steps 200 --warmup 10 --cpu-seconds 0 --host-gib 0 --no-tx"
for rep in 1 2; do
  for t in 0 1; do
    HVWS_TAIL=$t $S bench_${TAG}_c2_t${t}_$rep 200 $B --config c2
  done
done
for t in 0 1; do
  HVWS_TAIL=$t $S bench_${TAG}_c3_t${t} 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
done
$S trace_${TAG}_c2 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
