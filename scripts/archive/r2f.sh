set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="--cpu-seconds 0 --host-gib 0 --no-tx --steps 20"
for cfg in c2 c4; do
  for g in 0 16 32 64 128 256; do
    HVWS_PIPED_GRID=$g timeout -k 10 200 python bench.py --config $cfg $B > gpurun_out/r2f_${cfg}_g$g.json 2>gpurun_out/r2f_${cfg}_g$g.err || { echo "bench $cfg $g failed"; tail gpurun_out/r2f_${cfg}_g$g.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/r2f_${cfg}_g$g.json')); print('$cfg grid=$g', d['value'], d['ms_per_step'], d['unmask_ms_mean'], d['scan_path'], d.get('other_step_call_ms'))"
  done
done
