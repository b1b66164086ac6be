#!/bin/bash
# P3 bench under path / knob variants (stage times per step in each JSON line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-var}
i=0
while IFS= read -r envs; do
  [ -z "$envs" ] && continue
  i=$((i+1))
  env $envs timeout -k 10 240 python3 -u bench.py --steps 3 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  rc=$?
  echo "[$envs] rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e9,2), 'G', d['ms_per_step'], d['stage_ms_per_step'], d['counters']['carry'])" gpurun_out/${TAG}_$i.json 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done <<< "${VARIANTS}"
exit 0
