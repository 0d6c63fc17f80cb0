#!/bin/bash
# Round 2: unmask timing events attached to its dispatch (hipExtLaunchKernelGGL)
# instead of marker packets.  GPU suite, then c2 with the pipelined SPEC tail
# on the scan stream (HVWS_TAIL=0) and on the unmask stream (1), c3, c4, trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2h}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --steps 200 --warmup 10 --cpu-seconds 0 --host-gib 0 --no-tx"
for rep in 1 2; do
  for t in 0 1; do
    HVWS_TAIL=$t $S bench_${TAG}_c2_t${t}_$rep 200 $B --config c2
  done
done
$S bench_${TAG}_c2_serial 200 $B --config c2 --serial
$S bench_${TAG}_c4 200 $B --config c4 --segments 1024
$S bench_${TAG}_c3 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
$S trace_${TAG}_c2 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
