set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "pipeline or host" --timeout 200 --timeout-method thread > gpurun_out/r2h_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r2h_pytest.log; exit 1; }
tail -2 gpurun_out/r2h_pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/r2h_bench.json 2> gpurun_out/r2h_bench.err || { echo bench failed; tail gpurun_out/r2h_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2h_bench.json')); print(d['value'], d['roofline']['frac'], json.dumps(d['host_inclusive']))"
