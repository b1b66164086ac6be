#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-win}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_nfa.py tests/test_persistence.py tests/test_gpu_exchange.py tests/test_gpu_segscan.py tests/test_gpu_kat.py > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for c in S4-seq S4-not S4-seqplus; do
  SHD_NFA_DEBUG=1 timeout -k 10 120 python -u bench.py --config $c --steps 1 --warmup 0 --cpu-sample 1000 > gpurun_out/dbg_${TAG}_$c.json 2> gpurun_out/dbg_${TAG}_$c.err || exit 1
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-sample 200000 > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  r=$?; echo "bench $c rc=$r $(python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$c.json')); print(d['value']/1e6, 'M ev/s', d['ms_per_step'], d['stage_ms_per_step'], d['cpu_baseline']['value']/1e6)" 2>/dev/null)"
  [ $r -eq 0 ] || exit $r
done
