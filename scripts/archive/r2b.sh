set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "rejected_check or ends_monotone" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2b_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r2b_pytest.log; exit 1; }
tail -3 gpurun_out/r2b_pytest.log
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'tests')
import libhv_amd; libhv_amd.LIB_PATH='build/neg/libhvws.so'
import pytest
sys.exit(pytest.main(['tests/test_gpu_parity.py','-k','rejected_check','-q','-m','gpu','-p','no:cacheprovider']))
" > gpurun_out/r2b_neg.log 2>&1; echo "negative control rc=$? (expected nonzero)"; grep -E "assert|passed|failed|Error" gpurun_out/r2b_neg.log | head -20
