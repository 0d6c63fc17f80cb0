# round 3: FUSED parity subset, c2 bench FUSED auto vs off, rocprof kernel stats of the fused run
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3m
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "fused or batch_segments_with_carry or batch_every_cut or batch_empty or batch_configs_small or dense_tiny or speculative_table or pipelined_steps" \
  > gpurun_out/r3m/pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r3m/pytest.log; exit 1; }
tail -1 gpurun_out/r3m/pytest.log
B="--config c2 --steps 200 --warmup 5 --no-tx --host-gib 0 --cpu-seconds 0 --feed-conns 0 --dropin-reads 0"
for f in 2 0; do
  HVWS_FUSED=$f timeout -k 10 200 python -u bench.py $B > gpurun_out/r3m/c2_fused$f.json 2> gpurun_out/r3m/c2_fused$f.err || { echo "bench c2 failed"; tail -20 gpurun_out/r3m/c2_fused$f.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3m/c2_fused$f.json')); print('fused=$f', d['value'], d['ms_per_step'], d.get('scan_path'), d['unmask_ms_mean'], d['roofline']['kernel'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
HVWS_FUSED=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3m/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $B > $GRAFT_REPO_ROOT/gpurun_out/r3m/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3m/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r3m/prof -name "*kernel_stats.csv" -exec head -12 {} \;
