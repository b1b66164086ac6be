#!/bin/bash
# A/B the timestamp payload on the carry / pruning parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=tests/test_gpu_parity.py
run() { echo "== $*"; env "$@" timeout -k 10 120 python -u -m pytest $T -m gpu -q --timeout 100 --timeout-method thread \
  -p no:cacheprovider -k "pruned or 3-P3" 2>&1 | grep -E "^E |passed|failed" | head -20; }
run X=1 && run SHD_TS64=1
