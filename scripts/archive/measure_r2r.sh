#!/bin/bash
# Round 2: the table set's free event = the unmask's dispatch-attached stop
# event (no marker packet) vs a marker (HVWS_FREE_MARKER=1).  Parity suite,
# c2 / c4 A/B interleaved, c2 trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2r}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S parity_$TAG 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx"
for rep in 1 2; do
  for m in 0 1; do
    HVWS_FREE_MARKER=$m $S bench_${TAG}_c2_m${m}_$rep 200 $B --steps 200 --warmup 10 --config c2
    HVWS_FREE_MARKER=$m $S bench_${TAG}_c4_m${m}_$rep 200 $B --steps 100 --warmup 10 --config c4 --segments 1024
  done
done
$S trace_${TAG}_c2 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
