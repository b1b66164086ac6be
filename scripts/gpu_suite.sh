#!/bin/bash
# The GPU test suite in one process, selected files (FILES) or all; log under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-suite}
timeout -k 10 ${LIMIT:-1000} python -u -m pytest ${FILES:-tests} -m gpu -q -rs --timeout 180 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/${TAG}_pytest_gpu.log
exit $rc
