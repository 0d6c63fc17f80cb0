set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="--cpu-seconds 0 --host-gib 0 --no-tx --steps 20"
for cfg in c3 c2 c4; do
  for v in "" "--validate"; do
    tag=${cfg}$( [ -n "$v" ] && echo _val )
    timeout -k 10 200 python bench.py --config $cfg $B $v > gpurun_out/r2g_$tag.json 2>gpurun_out/r2g_$tag.err || { echo "bench $tag failed"; tail gpurun_out/r2g_$tag.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r2g_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['unmask_ms_mean'], d['scan_path'], d.get('other_step_call_ms'), d.get('validation'))"
  done
done
