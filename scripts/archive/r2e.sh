set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in c3 c2; do
timeout -k 10 300 python bench.py --config $cfg --sweep-unmask --cpu-seconds 0 --host-gib 0 --no-tx --steps 10 > gpurun_out/r2e_$cfg.json 2> gpurun_out/r2e_$cfg.err || { tail gpurun_out/r2e_$cfg.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r2e_$cfg.json'))
print('$cfg', d['value'], 'ceiling', d['stream_ceiling_GBps'])
for k,v in d['unmask_sweep_GBps'].items(): print('  ', k, v, d['stream_sweep_GBps'].get(k))
"
done
