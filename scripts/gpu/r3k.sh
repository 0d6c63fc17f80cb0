# round 3: FUSED path parity (fixed tail handling) and c2 bench fused vs SPEC
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3k
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "fused or batch_segments_with_carry or batch_every_cut or batch_empty or batch_configs_small or dense_tiny or speculative_table or pipelined_steps" \
  > gpurun_out/r3k/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL" gpurun_out/r3k/pytest.log | tail -5; tail -60 gpurun_out/r3k/pytest.log; exit 1; }
tail -3 gpurun_out/r3k/pytest.log
for f in 2 0; do
  HVWS_FUSED=$f timeout -k 10 200 python -u bench.py --config c2 --steps 200 --warmup 5 --no-tx --host-gib 0 --cpu-seconds 0 --feed-conns 0 --dropin-reads 0 > gpurun_out/r3k/c2_fused$f.json 2> gpurun_out/r3k/c2_fused$f.err || { echo "bench c2 failed"; tail -20 gpurun_out/r3k/c2_fused$f.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3k/c2_fused$f.json')); print('fused=$f', d['value'], d['ms_per_step'], d['scan_path'], d['unmask_ms_mean'], d['roofline']['frac'])"
done
