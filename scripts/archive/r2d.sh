set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2d_trace -o c2 -- python3 bench.py --config c2 --cpu-seconds 0 --host-gib 0 --no-tx --steps 8 --warmup 2 > gpurun_out/r2d_bench.json 2> gpurun_out/r2d_bench.err || { tail gpurun_out/r2d_bench.err; exit 1; }
find gpurun_out/r2d_trace -name "*kernel_trace.csv" | head
