#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-w2}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_segscan.py tests/test_gpu_kat.py tests/test_multi_query.py tests/test_gpu_parity.py -k "window or segscan or W2 or agg or group or kat or multi" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for c in W2-length W2-time; do
  timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/w2_${TAG}_$c.json 2>/dev/null || exit 1
  echo "$c $(python3 -c "import json; d=json.load(open('gpurun_out/w2_${TAG}_$c.json')); print(round(d['value']/1e9,2), 'G ev/s', d['stage_ms_per_step'])")"
done
