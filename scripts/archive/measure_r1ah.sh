#!/bin/bash
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
$S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
$S ah_c4s 200 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx
$S ah_c3s 200 python bench.py --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx --steps 6
$S ah_c3 300 python bench.py --cpu-seconds 0 --host-gib 4 --no-tx
