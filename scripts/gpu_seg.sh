#!/bin/bash
# Segmented-scan window aggregates: targeted GPU tests, then W2 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-seg}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_segscan.py "tests/test_gpu_parity.py::test_device_equals_oracle" \
    tests/test_gpu_parity.py::test_single_event_calls_match_oracle tests/test_gpu_parity.py::test_group_fold_long_segments \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for c in W2-length W2-time; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  r=$?; echo "bench $c rc=$r"; cat gpurun_out/bench_${TAG}_$c.json | head -c 1500; echo
  [ $r -eq 0 ] || exit $r
done
