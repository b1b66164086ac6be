#!/bin/bash
# A/B of library builds on one box: for each VARIANTS entry V, the P3 bench
# line and a kernel-stats pass with SHD_LIB=siddhi_amd/var_V.so.
#   VARIANTS="A B C" TAG=r06k bash scripts/gpu_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-var}
for V in ${VARIANTS}; do
  export SHD_LIB=$PWD/siddhi_amd/var_$V.so
  timeout -k 10 300 python3 -u bench.py --config ${CFG:-P3} > gpurun_out/${TAG}_${V}_bench.json 2> gpurun_out/${TAG}_${V}_bench.err
  rc=$?; echo "bench $V rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${V}_bench.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,3), 'G ev/s', d['ms_per_step'], d.get('stage_ms_per_step'), d.get('parity_prefix'))" gpurun_out/${TAG}_${V}_bench.json $V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_${V}_trace -o k -- python3 -u bench.py --config ${CFG:-P3} \
      --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/${TAG}_${V}_trace.log 2>&1
  rc=$?; echo "trace $V rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
