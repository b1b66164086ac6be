#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-nprof}
for c in S4-seq S4-seqplus S4-not; do
  SHD_LIB=siddhi_amd/libsiddhi_hip_prof.so SHD_NFA_DEBUG=1 timeout -k 10 200 python -u bench.py --config $c --steps 1 --warmup 0 --cpu-sample 1000 > gpurun_out/np_${TAG}_$c.json 2> gpurun_out/np_${TAG}_$c.err || exit 1
  echo "$c"; grep "shd nfa" gpurun_out/np_${TAG}_$c.err | tail -2
done
