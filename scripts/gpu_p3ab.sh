#!/bin/bash
# P3 variants A/B: default, sort path, unfused bucket prep, 16-bit hashed sort; P3-dense.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
run() {   # name, env...
  local name=$1; shift
  timeout -k 10 240 env "$@" python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} \
      > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err
  local r=$?
  echo "$name rc=$r $(python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_$name.json')); print(d['value']/1e9, d['ms_per_step'], d['stage_ms_per_step'])" 2>/dev/null)"
  return $r
}
run default X=1 && run sort SHD_NO_BUCKET=1 && run unfused SHD_BUCKET_UNFUSED=1 && run hash16 SHD_NO_BUCKET=1 SHD_HASH_BITS=16 && \
BENCH_ARGS="--config P3-dense" run dense X=1
