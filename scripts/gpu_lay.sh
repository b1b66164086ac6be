#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-lay}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_nfa.py tests/test_persistence.py tests/test_gpu_logical.py > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for c in S4-seq S4-seqplus S4-not S4P-seqplus; do
  for il in 0 1; do
    SHD_NFA_INTERLEAVE=$il timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-sample 1000 > gpurun_out/lay_${TAG}_${c}_$il.json 2>/dev/null || exit 1
    echo "$c interleave=$il $(python3 -c "import json; d=json.load(open('gpurun_out/lay_${TAG}_${c}_$il.json')); print(round(d['value']/1e6,1), 'M ev/s', d['stage_ms_per_step'])")"
  done
done
