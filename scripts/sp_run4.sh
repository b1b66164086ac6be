# pipelined lockstep + pre-decoded projection atoms: tests, then bench lines
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lockstep.py \
  tests/test_gpu_block_skip.py tests/test_gpu_fastpred.py tests/test_gpu_parity.py tests/test_gpu_logical.py \
  tests/test_gpu_share.py > gpurun_out/sp4_tests.log 2>&1
echo tests-ok; tail -2 gpurun_out/sp4_tests.log
for cfg in P3-dense P1 S4-or P3; do
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/sp4_$cfg.json 2> gpurun_out/sp4_$cfg.err
  echo $cfg; cut -c1-150 gpurun_out/sp4_$cfg.json
done
timeout -k 10 400 python bench.py --config M5 --events 100000000 --cpu-sample 0 > gpurun_out/sp4_M5.json 2> gpurun_out/sp4_M5.err
echo M5; cut -c1-150 gpurun_out/sp4_M5.json
