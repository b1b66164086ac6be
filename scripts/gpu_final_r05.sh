# round-5 closing check: the whole GPU suite with the current build
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rs > gpurun_out/r05b_pytest_gpu.log 2>&1
echo suite-ok; tail -2 gpurun_out/r05b_pytest_gpu.log
