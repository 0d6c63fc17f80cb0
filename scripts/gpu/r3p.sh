# round 3: k_fused kernel time (probe), then the fused parity subset
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3p
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u scripts/probe/fused_kernel.py c2 4096 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "fused or batch_segments_with_carry or batch_every_cut or batch_empty or batch_configs_small or dense_tiny or speculative_table or pipelined_steps" \
  > gpurun_out/r3p/pytest.log 2>&1 || { echo "pytest failed"; grep -E "^E |Error" gpurun_out/r3p/pytest.log | head -20; tail -3 gpurun_out/r3p/pytest.log; exit 1; }
tail -1 gpurun_out/r3p/pytest.log
