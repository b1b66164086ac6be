# NFA lane kernel occupancy check: its tests, then the S4 NFA configs
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nfa.py > gpurun_out/nfa_occ_tests.log 2>&1
echo tests-ok; tail -1 gpurun_out/nfa_occ_tests.log
for cfg in S4-seq S4-seqplus S4P-seqplus; do
  timeout -k 10 300 python bench.py --config $cfg --cpu-sample 0 > gpurun_out/nfa_occ_$cfg.json 2> gpurun_out/nfa_occ_$cfg.err
  echo $cfg; cut -c1-130 gpurun_out/nfa_occ_$cfg.json
done
