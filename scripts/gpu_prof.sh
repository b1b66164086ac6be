#!/bin/bash
# rocprofv3 kernel stats (csv) of the default bench + HBM traffic PMC passes on one 25M-event push.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${BENCH_ARGS:-}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$TAG -o p3 -- python3 -u bench.py --steps 2 --warmup 1 --cpu-sample 0 $ARGS \
    > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_$TAG.log; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C -f csv -d gpurun_out/pmc_${C}_$TAG -o p3 -- python3 -u bench.py --steps 1 --warmup 0 \
      --cpu-sample 0 --events 25000000 $ARGS > gpurun_out/pmc_${C}_$TAG.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; tail -1 gpurun_out/pmc_${C}_$TAG.log
  [ $rc -eq 0 ] || exit $rc
done
find gpurun_out/prof_$TAG gpurun_out/pmc_*_$TAG -name "*.csv" | head -20
