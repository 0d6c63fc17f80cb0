#!/bin/bash
# round 3 final tree (worker off by default, drop-in leg opt-in): GPU suite,
# smoke, the default bench three times, the default bench under rocprofv3,
# the drop-in leg alone; stops at the first crash or hang
set -u
S=scripts/gpu_step.sh
TAG=${1:-r3ag}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONFAULTHANDLER=1
rm -f gpurun_out/.stop
$S pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ -f gpurun_out/.stop ] && exit 1
$S smoke_$TAG 120 python3 -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  $S bench${i}_$TAG 200 python3 bench.py
  [ -f gpurun_out/.stop ] && exit 1
done
$S trace_${TAG}_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG}_c3 -o run --output-format csv -- python3 bench.py
[ -f gpurun_out/.stop ] && exit 1
$S dropin_$TAG 200 python3 scripts/bench_dropin.py 2000
