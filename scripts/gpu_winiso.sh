#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-iso}
SHD_NFA_DEBUG=1 timeout -k 10 400 python -u -m pytest -x -v -s --timeout 100 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_nfa.py -k "window_lanes" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Timeout" gpurun_out/pytest_$TAG.log | tail -5; tail -5 gpurun_out/pytest_$TAG.log
exit $rc
