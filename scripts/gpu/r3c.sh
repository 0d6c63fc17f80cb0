# round 3: device memory probe; resident worker tests; drop-in latency
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3c
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u scripts/probe/mem_probe.py > gpurun_out/r3c/mem_probe.log 2>&1 || { echo "mem probe failed"; tail -20 gpurun_out/r3c/mem_probe.log; exit 1; }
cat gpurun_out/r3c/mem_probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3c/door.log 2>&1 || { echo "door tests failed"; tail -60 gpurun_out/r3c/door.log; exit 1; }
tail -12 gpurun_out/r3c/door.log
timeout -k 10 200 python -u scripts/bench_dropin.py > gpurun_out/r3c/dropin.json 2> gpurun_out/r3c/dropin.err || { echo "dropin failed"; tail -20 gpurun_out/r3c/dropin.err; exit 1; }
cat gpurun_out/r3c/dropin.json
