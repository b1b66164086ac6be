#!/bin/bash
# rocprofv3 kernel stats of one short bench run per variant (VARIANTS="name:ENV=VAL,ENV2=VAL name2:" ...)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-kp}
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; envs=${v#*:}
  for e in ${envs//,/ }; do export "$e"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kp_${TAG}_$name -o k -- python3 -u bench.py --steps 1 --warmup 1 \
      --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/kp_${TAG}_$name.log 2>&1
  rc=$?; echo "== $name ($envs) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/kp_${TAG}_$name.log
  python3 - gpurun_out/kp_${TAG}_$name/k_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print("%-60s %5s %9.1f us %6s" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"]))
PY
  for e in ${envs//,/ }; do unset "${e%%=*}"; done
done
