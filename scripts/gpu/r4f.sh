#!/bin/bash
# round 4: the worker's run-length position chase (door tests, phases, per-call
# latency); then reproduce round 3's bench hang with round 3's own build (commit
# 0db4e5f, built into build/r3tree: worker on by default, the early-return
# park, drop-in leg on), every run under a watchdog that prints every thread's
# Python and native stacks after 60 s; then the current tree's bench with the
# drop-in leg and the worker on, twice
set -u
S=scripts/gpu_step.sh
TAG=${1:-r4f}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_$TAG 300 python -u -m pytest tests/test_gpu_door.py -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S door_phases_$TAG 120 python3 scripts/probe/door_phases.py 2000
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
[ -f gpurun_out/.stop ] && exit 1
for i in 1 2 3 4; do
  HVWS_BENCH_WATCHDOG=0 $S r3bench_${i}_$TAG 240 python3 scripts/probe/watchdog_run.py 60 build/r3tree/bench.py
  [ -f gpurun_out/.stop ] && exit 1
done
for i in 1 2; do
  HVWS_DOOR=1 HVWS_BENCH_WATCHDOG=60 $S bench_dropin_${i}_$TAG 300 python3 bench.py --dropin-reads 2000
  [ -f gpurun_out/.stop ] && exit 1
done
exit 0
