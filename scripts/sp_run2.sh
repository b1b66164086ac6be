# split-f2 kinds + NFA fast filters: parity tests, then bench lines
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lockstep.py \
  tests/test_gpu_block_skip.py tests/test_gpu_nfa.py tests/test_gpu_parity.py tests/test_gpu_kat.py > gpurun_out/sp2_tests.log 2>&1
echo tests-ok; tail -2 gpurun_out/sp2_tests.log
for cfg in P3-dense P3 S4-seq S4-seqplus S4P-seqplus; do
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/sp2_$cfg.json 2> gpurun_out/sp2_$cfg.err
  echo $cfg; cut -c1-160 gpurun_out/sp2_$cfg.json
done
