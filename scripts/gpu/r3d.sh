# round 3: memory fix check; resident worker tests; drop-in latency; configs incl. c5 ranks
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3d
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u scripts/probe/mem_probe.py > gpurun_out/r3d/mem_probe.log 2>&1 || { echo "mem probe failed"; tail -20 gpurun_out/r3d/mem_probe.log; exit 1; }
cat gpurun_out/r3d/mem_probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_door.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3d/door.log 2>&1 || { echo "door tests failed"; tail -60 gpurun_out/r3d/door.log; exit 1; }
tail -12 gpurun_out/r3d/door.log
timeout -k 10 200 python -u scripts/bench_dropin.py > gpurun_out/r3d/dropin.json 2> gpurun_out/r3d/dropin.err || { echo "dropin failed"; tail -20 gpurun_out/r3d/dropin.err; exit 1; }
cat gpurun_out/r3d/dropin.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3d/configs.log 2>&1 || { echo "config tests failed"; tail -40 gpurun_out/r3d/configs.log; exit 1; }
tail -16 gpurun_out/r3d/configs.log
