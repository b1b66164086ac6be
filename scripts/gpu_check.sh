#!/bin/bash
# Iteration check on one GPU: selected GPU tests, the P3 bench line and a
# rocprofv3 kernel-stats pass of the same bench command.
#   TAG=r06b TESTS="tests/test_gpu_fused_sort.py" bash scripts/gpu_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-chk}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v -rs --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for C in ${CONFIGS:-P3}; do
  [ "$C" = none ] && continue
  timeout -k 10 300 python3 -u bench.py --config $C ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_$C.json 2> gpurun_out/${TAG}_bench_$C.err
  rc=$?; echo "bench $C rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench_$C.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e9,3), 'G ev/s', d['ms_per_step'], d.get('stage_ms_per_step'), d.get('parity_prefix'), (d.get('derived_check') or {}).get('equal'))" gpurun_out/${TAG}_bench_$C.json
done
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_trace -o k -- python3 -u bench.py --config ${PROF_CFG:-P3} \
      --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/${TAG}_trace.log 2>&1
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/${TAG}_trace/k_kernel_stats.csv <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:16]:
    print(x['Name'][:60].ljust(60), x['Calls'], round(float(x['AverageNs']) / 1e3, 1), x['Percentage'])
PY
fi
exit 0
