#!/bin/bash
# Adaptive unmask pieces: parity (pipelined cases), c4 / c2 / c3 / c4 one stream.
set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
#$S pytest_parity 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
$S ad_c4 200 python bench.py --config c4 --segments 1024 --cpu-seconds 0 --host-gib 0 --no-tx
$S ad_c2 200 python bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx
$S ad_c3 200 python bench.py --cpu-seconds 0 --host-gib 0 --no-tx --steps 6
$S ad_c4s 200 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx
HVWS_UNMASK_PIECES=4 $S ad_c4s_p4 200 python bench.py --config c4 --segments 1 --cpu-seconds 0 --host-gib 0 --no-tx
