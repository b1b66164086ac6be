set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bucket.py > gpurun_out/g3_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/g3_pytest.log
SHD_DEBUG_BUCKET=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/g3_bench.json 2> gpurun_out/g3_bench.err
echo "bench rc=$?" >> gpurun_out/g3_bench.err
SHD_BUCKET_UNFUSED=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/g3_bench_unfused.json 2>> gpurun_out/g3_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g3_prof -o g3 -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/g3_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/g3_prof.log
