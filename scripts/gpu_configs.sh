#!/bin/bash
# One bench line per BASELINE config shape (P1, W2-length, W2-time, S4-*, M5 sample) + P3 as rank 1's key slice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-cfg}
for c in ${CONFIGS:-P1 W2-length W2-time S4-or S4P-seqplus}; do
  timeout -k 10 300 python3 -u bench.py --config $c --cpu-sample ${CPU:-0} > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err
  rc=$?; echo "== $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d.get('stage_ms_per_step'), (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/${TAG}_$c.json
done
if [ -n "${M5_EVENTS:-}" ]; then
  timeout -k 10 400 python3 -u bench.py --config M5 --events $M5_EVENTS --steps 1 --warmup 1 > gpurun_out/${TAG}_M5.json 2> gpurun_out/${TAG}_M5.err
  rc=$?; echo "== M5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['query_events_per_s'], d['ms_per_step'], d['stage_ms_per_step_rank0'])" gpurun_out/${TAG}_M5.json
fi
if [ -n "${RANK1:-}" ]; then
  RANK=1 timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > gpurun_out/${TAG}_P3_rank1.json 2>&1
  rc=$?; echo "== P3 as rank 1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['stage_ms_per_step'])" gpurun_out/${TAG}_P3_rank1.json
fi
