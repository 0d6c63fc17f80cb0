#!/bin/bash
# Round 2: in-place stream rate per buffer (3 x 64 GiB), and the default bench.
set -u
S=scripts/gpu_step.sh
TAG=${1:-r2v}
export TMPDIR=/tmp
rm -f gpurun_out/.stop
$S bufprobe_$TAG 300 python3 scripts/buffer_probe.py
$S bench_$TAG 400 python3 bench.py --cpu-seconds 0 --host-gib 0
