#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py > gpurun_out/pytest_p3q.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_p3q.log
timeout -k 10 200 python -u bench.py --config P3 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/p3q.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/p3q.json')); print(round(d['value']/1e9,2), 'G ev/s', d['stage_ms_per_step'])"
