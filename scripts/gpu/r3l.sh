# round 3: c2 bench, FUSED auto vs off, plus a rocprof kernel trace of the fused run
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3l
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="--config c2 --steps 200 --warmup 5 --no-tx --host-gib 0 --cpu-seconds 0 --feed-conns 0 --dropin-reads 0"
for f in 2 0; do
  HVWS_FUSED=$f timeout -k 10 200 python -u bench.py $B > gpurun_out/r3l/c2_fused$f.json 2> gpurun_out/r3l/c2_fused$f.err || { echo "bench c2 failed"; tail -20 gpurun_out/r3l/c2_fused$f.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3l/c2_fused$f.json')); print('fused=$f', d['value'], d['ms_per_step'], d.get('scan_path'), d['roofline'])"
done
cd /tmp && export TMPDIR=/tmp
HVWS_FUSED=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3l/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $B > $GRAFT_REPO_ROOT/gpurun_out/r3l/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3l/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r3l/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
