#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config P3 --steps 3 --warmup 1 --cpu-sample 0 --sweep-batches 5000000,10000000,20000000,25000000,50000000 > gpurun_out/p3batch.json 2> gpurun_out/p3batch.err || exit 1
grep sweep_batch gpurun_out/p3batch.err
