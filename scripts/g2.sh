set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bucket.py tests/test_gpu_fallback.py tests/test_gpu_parity.py > gpurun_out/g2_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/g2_pytest.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/g2_bench.json 2> gpurun_out/g2_bench.err
echo "bench rc=$?" >> gpurun_out/g2_bench.err
