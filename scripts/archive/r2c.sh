set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="--cpu-seconds 0 --host-gib 0 --no-tx --steps 20"
for cfg in c2 c4; do
  for pr in 0 1; do
    HVWS_SCAN_PRIORITY=$pr timeout -k 10 200 python bench.py --config $cfg $B > gpurun_out/r2c_${cfg}_p$pr.json 2>gpurun_out/r2c_${cfg}_p$pr.err || { echo "bench $cfg $pr failed"; tail gpurun_out/r2c_${cfg}_p$pr.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r2c_${cfg}_p$pr.json')); print('$cfg prio=$pr', d['value'], d['ms_per_step'], d['unmask_ms_mean'], d['scan_path'], d.get('other_step_call_ms'))"
  done
done
