# round 3: transmit k_build_id -- parity, then c2/c3 transmit legs (same-offset vs general)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3q
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3q/pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |Error" gpurun_out/r3q/pytest.log | head -20; tail -3 gpurun_out/r3q/pytest.log; exit 1; }
tail -1 gpurun_out/r3q/pytest.log
for id in 1 0; do
  HVWS_BUILD_ID=$id timeout -k 10 200 python -u bench.py --config c2 --steps 20 --warmup 2 --host-gib 0 --cpu-seconds 0 --feed-conns 0 --dropin-reads 0 > gpurun_out/r3q/c2_id$id.json 2> gpurun_out/r3q/c2_id$id.err || { echo "bench failed"; tail -5 gpurun_out/r3q/c2_id$id.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3q/c2_id$id.json')); print('c2 id=$id', d['tx'])"
done
