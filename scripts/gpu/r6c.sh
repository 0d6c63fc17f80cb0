#!/bin/bash
# r6c: the GPU suite on round 6's first tree (lagged stepper and RUN geometries
# removed, RUN regression tests, full-size c2 RUN digests), then r6b's exit probes.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_run_r6c 300 python -u -m pytest tests/test_gpu_run.py tests/test_gpu_configs.py -k "run or config2" -x -v --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S pytest_gpu_r6c 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
bash scripts/gpu/r6b.sh
