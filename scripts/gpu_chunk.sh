#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-chunk}
for c in S4-seq S4-seqplus; do
  for ch in 4 8 16 32; do
    SHD_NFA_CHUNK=$ch timeout -k 10 120 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-sample 1000 > gpurun_out/ch_${TAG}_${c}_$ch.json 2>/dev/null || exit 1
    echo "$c chunk=$ch $(python3 -c "import json; d=json.load(open('gpurun_out/ch_${TAG}_${c}_$ch.json')); print(round(d['value']/1e6,1), 'M ev/s', d['stage_ms_per_step'])")"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o s4seq -- python3 bench.py --config S4-seq --steps 3 --warmup 1 --cpu-sample 1000 > gpurun_out/prof_$TAG.log 2>&1 || exit 1
python3 scripts/rocpd_stats.py gpurun_out/prof_$TAG > gpurun_out/prof_${TAG}_stats.txt 2>&1; head -12 gpurun_out/prof_${TAG}_stats.txt
