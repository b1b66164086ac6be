#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for hb in 0 16 8; do
  if [ $hb = 0 ]; then unset SHD_HASH_BITS; else export SHD_HASH_BITS=$hb; fi
  timeout -k 10 200 python -u bench.py --config P3 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/p3h_$hb.json 2>/dev/null || exit 1
  echo "hash_bits=$hb $(python3 -c "import json; d=json.load(open('gpurun_out/p3h_$hb.json')); print(round(d['value']/1e9,2), 'G ev/s', d['stage_ms_per_step'], d['counters'])")"
done
