#!/bin/bash
# Round-3 check of the HIP re-route passes: parity tests, the round-robin
# bench path at N = 1 (HIP route vs the round-2 torch route), and a kernel
# trace of P3-dense.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03n}
timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests/test_gpu_route.py} -x -v -rs --timeout 120 --timeout-method thread \
  > gpurun_out/route_$T.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/route_$T.log; exit 1; }
tail -3 gpurun_out/route_$T.log
timeout -k 10 300 python3 -u bench.py --input roundrobin --steps 3 --warmup 1 --cpu-sample 0 \
  > gpurun_out/rr_hip_$T.json 2> gpurun_out/rr_hip_$T.err || { echo "rr hip rc=$?"; tail -20 gpurun_out/rr_hip_$T.err; exit 1; }
SHD_ROUTE_TORCH=1 timeout -k 10 300 python3 -u bench.py --input roundrobin --steps 3 --warmup 1 --cpu-sample 0 \
  > gpurun_out/rr_torch_$T.json 2> gpurun_out/rr_torch_$T.err || { echo "rr torch rc=$?"; exit 1; }
for f in rr_hip rr_torch; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e9,3), 'G', d['ms_per_step'], d.get('stage_ms_per_step'))" gpurun_out/${f}_$T.json
done
if [ -n "${DENSE:-1}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${T}_dense -o k -- python3 -u bench.py \
    --config P3-dense --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/${T}_dense.log 2>&1 || { echo "dense rc=$?"; exit 1; }
  f=$(ls gpurun_out/${T}_dense/*/k_kernel_stats.csv 2>/dev/null || ls gpurun_out/${T}_dense/k_kernel_stats.csv)
  head -14 $f | cut -c1-160
fi
exit 0
