set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2a_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r2a_pytest.log; exit 1; }
tail -3 gpurun_out/r2a_pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/r2a_bench.json 2> gpurun_out/r2a_bench.err || { echo bench failed; tail gpurun_out/r2a_bench.err; exit 1; }
cat gpurun_out/r2a_bench.json
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'tests')
import libhv_amd; libhv_amd.LIB_PATH='build/neg/libhvws.so'
import pytest
sys.exit(pytest.main(['tests/test_gpu_parity.py','-k','rejected_check','-x','-q','-m','gpu','-p','no:cacheprovider']))
" > gpurun_out/r2a_neg.log 2>&1; echo "negative control rc=$? (expected nonzero)"; tail -15 gpurun_out/r2a_neg.log
