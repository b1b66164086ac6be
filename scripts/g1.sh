set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fallback.py tests/test_gpu_parity.py tests/test_persistence.py > gpurun_out/g1_pytest.log 2>&1
echo "rc=$?" >> gpurun_out/g1_pytest.log
