#!/bin/bash
# Round 2: one-walk SPEC/SLACK passes without the k_verify pair and
# k_head<true> (adaptive), unmask-only timing markers in pipelined steps.
# Full GPU suite, then c2/c4 with the verify pair forced (1) and adaptive (-1),
# c3 default, and a c2 kernel trace.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2e}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
B="python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx"
for cfg in c2 c4; do
  seg=4096; [ $cfg = c4 ] && seg=1024
  for v in 1 -1; do
    HVWS_WALK_VERIFY=$v $S bench_${TAG}_${cfg}_v$v 200 $B --config $cfg --segments $seg
    HVWS_WALK_VERIFY=$v $S bench_${TAG}_${cfg}_v${v}_serial 200 $B --config $cfg --segments $seg --serial
  done
done
$S bench_${TAG}_c3 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
$S trace_${TAG}_c2 300 rocprofv3 --kernel-trace -d gpurun_out/trace_${TAG}_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 0 --host-gib 0 --no-tx
