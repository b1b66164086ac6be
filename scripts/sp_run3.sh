# pipelined lockstep walk: its tests, then the dense bench line
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lockstep.py \
  tests/test_gpu_block_skip.py > gpurun_out/sp3_tests.log 2>&1
echo tests-ok; tail -2 gpurun_out/sp3_tests.log
timeout -k 10 300 python bench.py --config P3-dense > gpurun_out/sp3_P3-dense.json 2> gpurun_out/sp3.err
cut -c1-160 gpurun_out/sp3_P3-dense.json
