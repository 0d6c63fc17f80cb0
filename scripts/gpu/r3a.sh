# round 3, first pass: advisor fixes, c3/c5 reference digests, multi-rank bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3a
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "over_host_record_area or nested_feed or free_from_callback or rx_reads or feed_many or feeder or threads or test_gpu_configs" \
  > gpurun_out/r3a/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3a/pytest.log; exit 1; }
tail -3 gpurun_out/r3a/pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err || { echo bench failed; tail gpurun_out/r3a/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3a/bench.json')); print(d['value'], d['roofline']['frac'], json.dumps(d['verified']), json.dumps(d['host_inclusive']['aggregate']), json.dumps(d['cpu_baseline']['multi_thread']), d['cpu_baseline']['cpu_model'])"
HVWS_BENCH_DEVICE=0 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 > gpurun_out/r3a/bench_n2.json 2> gpurun_out/r3a/bench_n2.err || { echo bench n2 failed; tail -30 gpurun_out/r3a/bench_n2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3a/bench_n2.json')); print(d['value'], json.dumps(d['timing']), json.dumps(d['host_inclusive']['aggregate']), json.dumps(d['host_inclusive']['per_rank']), json.dumps(d['verified']))"
