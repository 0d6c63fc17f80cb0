# round 3: worker with ordinary pinned data areas + serial walk prefix (k_door, k_small)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3g
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u scripts/probe/door_phases.py 2000 > gpurun_out/r3g/door_phases.json 2>&1 || { echo "phases failed"; tail -20 gpurun_out/r3g/door_phases.json; exit 1; }
cat gpurun_out/r3g/door_phases.json
timeout -k 10 200 python -u scripts/bench_dropin.py > gpurun_out/r3g/dropin.json 2> gpurun_out/r3g/dropin.err || { echo "dropin failed"; tail -20 gpurun_out/r3g/dropin.err; exit 1; }
cat gpurun_out/r3g/dropin.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "door or feed_many or feeder or rx_reads or threads or messages or execute or decode or small or batch_configs or over_host_record_area" \
  > gpurun_out/r3g/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3g/pytest.log; exit 1; }
tail -3 gpurun_out/r3g/pytest.log
