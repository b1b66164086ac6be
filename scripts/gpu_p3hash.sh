#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-p3}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_exchange.py tests/test_gpu_logical.py > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for v in fused unfused hash16; do
  unset SHD_SORT_UNFUSED SHD_HASH_BITS
  [ $v = unfused ] && export SHD_SORT_UNFUSED=1
  [ $v = hash16 ] && export SHD_SORT_UNFUSED=1 SHD_HASH_BITS=16
  timeout -k 10 200 python -u bench.py --config P3 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/p3h_${TAG}_$v.json 2>/dev/null || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/p3h_${TAG}_$v.json')); print(round(d['value']/1e9,2), 'G ev/s', d['stage_ms_per_step'], d['counters']['matches'])")"
done
