#!/bin/bash
# The closing pass of a round on one GPU box: the whole GPU suite, smoke, the
# default bench line, the RUN / SPEC c2 A/B and transmit lines, and the
# kernel-trace profile of the default bench, every step under its own limit
# (scripts/gpu_step.sh: any failure ends the call).
#   gpurun --timeout 1200 -- 'bash scripts/gpu/closing.sh r6z'
set -u
S=scripts/gpu_step.sh
TAG=${1:-closing}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 300 python3 scripts/smoke_run.py
[ -f gpurun_out/.stop ] && exit 1
$S bench_$TAG 400 python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
for run in 1 0; do
  $S c2_run${run}_$TAG 180 env HVWS_RUN=$run python3 bench.py --config c2 --steps 200 --warmup 10 --no-tx --feed-conns 0 --dropin-reads 0 --host-gib 0 --cpu-seconds 0
  [ -f gpurun_out/.stop ] && exit 1
done
for cfg in c2 c3 c4; do
  CONFIG=$cfg $S tx_${cfg}_$TAG 200 python3 scripts/bench_tx.py
  [ -f gpurun_out/.stop ] && exit 1
done
# c4 as one stream (the frame sieve), then the traced default bench with every leg on,
# the drop-in's resident worker included (its HSA queue is destroyed at exit)
$S c4_one_$TAG 240 python3 bench.py --config c4 --segments 1 --steps 40 --warmup 5 --no-tx --feed-conns 0 --dropin-reads 0 --host-gib 0 --cpu-seconds 0
[ -f gpurun_out/.stop ] && exit 1
$S kt_$TAG 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o kt -- python3 bench.py
exit 0
