#!/bin/bash
# Targeted GPU session: selected tests (-k / files in $TESTS), optional
# diagnostics ($DIAG: python scripts), optional P3 bench ($BENCH=1) and
# rocprofv3 kernel stats ($PROF=1).  Stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-q}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v -rs --timeout 180 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_$TAG.log | tail -40
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -qE "illegal memory access|APERTURE_VIOLATION|HSA_STATUS_ERROR|Memory access fault" gpurun_out/pytest_$TAG.log; then echo "GPU fault seen: stopping"; exit 3; fi
fi
for d in ${DIAG:-}; do
  timeout -k 10 300 python -u $d > gpurun_out/diag_${TAG}_$(basename $d .py).log 2>&1
  r=$?; echo "diag $d rc=$r"; tail -30 gpurun_out/diag_${TAG}_$(basename $d .py).log
  [ $r -eq 0 ] || exit $r
done
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  r3=$?; echo "bench rc=$r3"; tail -c 3000 gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
  [ $r3 -eq 0 ] || exit $r3
fi
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o p3 -- python3 -u bench.py --steps 2 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} \
      > gpurun_out/prof_$TAG.log 2>&1
  r4=$?; echo "rocprof rc=$r4"; tail -2 gpurun_out/prof_$TAG.log
  [ $r4 -eq 0 ] || exit $r4
fi
exit 0
