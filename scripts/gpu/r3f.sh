# round 3: door phase stamps; configs incl. c5 ranks (buffer reuse); N=2 rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3f
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u scripts/probe/door_phases.py 2000 > gpurun_out/r3f/door_phases.json 2>&1 || { echo "phases failed"; tail -20 gpurun_out/r3f/door_phases.json; exit 1; }
cat gpurun_out/r3f/door_phases.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3f/configs.log 2>&1 || { echo "config tests failed"; tail -40 gpurun_out/r3f/configs.log; exit 1; }
tail -16 gpurun_out/r3f/configs.log
HVWS_BENCH_DEVICE=0 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 > gpurun_out/r3f/bench_n2.json 2> gpurun_out/r3f/bench_n2.err || { echo bench n2 failed; tail -30 gpurun_out/r3f/bench_n2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3f/bench_n2.json')); print(d['value'], json.dumps(d['timing']), json.dumps(d['host_inclusive']['aggregate']), json.dumps(d['host_inclusive']['per_rank']), json.dumps(d['verified']), json.dumps(d.get('drop_in')))"
