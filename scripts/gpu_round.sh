#!/bin/bash
# One GPU session: gpu tests, smoke, full P3 bench, rocprofv3 kernel stats.
# Stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 180 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if grep -qE "illegal memory access|APERTURE_VIOLATION|HSA_STATUS_ERROR|Memory access fault" gpurun_out/pytest_gpu_$TAG.log; then echo "GPU fault seen: stopping"; exit 3; fi
[ "${SKIP_BENCH:-0}" = "1" ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
r2=$?; echo "smoke rc=$r2"; tail -3 gpurun_out/smoke_$TAG.log
[ $r2 -eq 0 ] || exit $r2
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
r3=$?; echo "bench rc=$r3"; tail -c 2500 gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
[ $r3 -eq 0 ] || exit $r3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o p3 -- python3 -u bench.py --steps 2 --warmup 1 --cpu-sample 0 \
    > gpurun_out/prof_$TAG.log 2>&1
r4=$?; echo "rocprof rc=$r4"; tail -2 gpurun_out/prof_$TAG.log
find gpurun_out/prof_$TAG -name "*stats*.csv" | head
exit $rc
