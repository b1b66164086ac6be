# split-f2 check: parity tests, then bench lines for the pattern configs
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lockstep.py \
  tests/test_gpu_block_skip.py tests/test_gpu_parity.py tests/test_gpu_fastpred.py tests/test_gpu_logical.py > gpurun_out/sp_tests.log 2>&1
echo tests-ok; tail -2 gpurun_out/sp_tests.log
for cfg in P3-dense P3 P1; do
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/sp_$cfg.json 2> gpurun_out/sp_$cfg.err
  echo $cfg; cut -c1-200 gpurun_out/sp_$cfg.json
done
SHD_LOCKSTEP=1 timeout -k 10 300 python bench.py --config P3-dense > gpurun_out/sp_ls_P3-dense.json 2> gpurun_out/sp_ls.err
echo ls; cut -c1-200 gpurun_out/sp_ls_P3-dense.json
