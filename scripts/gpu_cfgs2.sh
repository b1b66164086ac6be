#!/bin/bash
# Round-2 config lines: P3 (default and round-robin input), S4 window lanes, W2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-c2}
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/cfg_${TAG}_$nm.json 2> gpurun_out/cfg_${TAG}_$nm.err
  local r=$?
  echo "$nm rc=$r $(python3 -c "import json; d=json.load(open('gpurun_out/cfg_${TAG}_$nm.json')); print(round(d['value']/1e6,1), 'M ev/s', d['ms_per_step'], d.get('stage_ms_per_step'), (d.get('cpu_baseline') or {}).get('value'))" 2>/dev/null)"
  return $r
}
run P3rr --config P3 --input roundrobin --steps 3 --warmup 1 --cpu-sample 0 &&
run S4-seq --config S4-seq --steps 3 --warmup 1 --cpu-sample 200000 &&
run S4-seqplus --config S4-seqplus --steps 3 --warmup 1 --cpu-sample 200000 &&
run S4-not --config S4-not --steps 2 --warmup 1 --cpu-sample 200000 &&
run S4P-seqplus --config S4P-seqplus --steps 3 --warmup 1 --cpu-sample 200000 &&
run W2-length --config W2-length --steps 3 --warmup 1 --cpu-sample 200000 &&
run W2-time --config W2-time --steps 3 --warmup 1 --cpu-sample 200000
