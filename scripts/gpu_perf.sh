#!/bin/bash
# Parity (pattern + NFA + window) then a micro-batch sweep and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-perf}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nfa.py tests/test_gpu_fastpred.py -m gpu -q --timeout 180 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --sweep-batches ${SWEEP:-2000000,4000000,8000000,12500000,25000000} \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; grep sweep_batch gpurun_out/bench_$TAG.err | cut -c1-400; tail -c 1500 gpurun_out/bench_$TAG.json
exit $rc
