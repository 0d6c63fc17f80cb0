#!/bin/bash
# Round 2: single-block scan-chain kernels (offsets, checks) as 256-thread
# workgroups.  Parity suite, then c2 / c4 / c4 one stream pipelined.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2q}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S parity_$TAG 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --cpu-seconds 0 --host-gib 0 --no-tx"
for rep in 1 2; do
  $S bench_${TAG}_c2_$rep 200 $B --steps 200 --warmup 10 --config c2
  $S bench_${TAG}_c4_$rep 200 $B --steps 100 --warmup 10 --config c4 --segments 1024
done
$S bench_${TAG}_c4seg1 300 $B --config c4 --segments 1 --steps 40 --warmup 5
$S trace_${TAG}_c2 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
