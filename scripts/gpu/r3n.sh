# round 3: k_fused probe variants at c2 (kernel times; dbg variants give wrong bytes by design)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3n
export HSA_ENABLE_IPC_MODE_LEGACY=0
for d in 0 64 128 134 198; do
  HVWS_FUSED_DBG=$d timeout -k 10 120 python -u scripts/probe/fused_kernel.py c2 4096 2>&1 | grep -v amdgpu.ids | grep fused=1 || exit 1
done
