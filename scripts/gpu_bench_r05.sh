# round-5 closing bench lines: smoke, the headline P3 line, P3-dense, M5 at 100 M events
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b_smoke.log 2>&1
echo smoke-ok
for cfg in P3 P3-dense; do
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/r05b_bench_$cfg.json 2> gpurun_out/r05b_bench_$cfg.err
  echo $cfg; cut -c1-150 gpurun_out/r05b_bench_$cfg.json
done
# k_filter_items probes (timing only, results invalid): 1 = no look-back wait, 2 = no item writes
for pr in 0 1 2; do
  SHD_FI_PROBE=$pr timeout -k 10 300 python bench.py --config W2-length --cpu-sample 0 > gpurun_out/r05b_fi$pr.json 2> gpurun_out/r05b_fi$pr.err || true
  echo probe $pr; cut -c1-120 gpurun_out/r05b_fi$pr.json
done
