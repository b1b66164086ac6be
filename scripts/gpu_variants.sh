#!/bin/bash
# Bench stage times of the in-tree library and each bench_bin/*.so timing variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in siddhi_amd/libsiddhi_hip.so bench_bin/*.so; do
  echo "== $lib"
  SHD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/var.json 2> gpurun_out/var.err \
    || { echo "rc=$?"; tail -3 gpurun_out/var.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/var.json'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); print(round(d['value']/1e9,2), d['ms_per_step'], d['stage_ms_per_step'])
"
done
