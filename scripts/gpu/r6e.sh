#!/bin/bash
# r6e: the worker on its own HSA queue -- door tests, the child-exit tests,
# the exit probes traced (the r6a crash), 100 door_first processes, the GPU
# suite, the drop-in latency, and the traced default bench with the drop-in leg on.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_door_r6e 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S exit_kt_r6e 90 rocprofv3 --kernel-trace --stats -d gpurun_out/r6e_kt_exit -o kt -- python3 scripts/probe/exit_probe.py kt_r6e
[ -f gpurun_out/.stop ] && exit 1
EXIT_PROBE_RELEASE=1 $S exit_rel_kt_r6e 90 rocprofv3 --kernel-trace --stats -d gpurun_out/r6e_kt_rel -o kt -- python3 scripts/probe/exit_probe.py rel_r6e
[ -f gpurun_out/.stop ] && exit 1
$S door_first_r6e 400 bash scripts/probe/door_first.sh run 100
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_r6e 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S dropin_r6e 200 python3 scripts/bench_dropin.py
[ -f gpurun_out/.stop ] && exit 1
$S kt_bench_r6e 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6e_kt_bench -o kt -- python3 bench.py
exit 0
