#!/bin/bash
# One GPU session: gpu tests, smoke, a reduced bench.  Stops at the first
# fault / abort / timeout (exit codes other than 0 or 1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if grep -qE "illegal memory access|APERTURE_VIOLATION|HSA_STATUS_ERROR" gpurun_out/pytest_gpu.log; then echo "GPU fault seen: stopping"; exit 3; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --events ${BENCH_EVENTS:-10000000} --keys ${BENCH_KEYS:-1000000} \
    --cpu-sample 200000 > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_small.log
exit $rc
