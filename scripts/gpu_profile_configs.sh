#!/bin/bash
# Build-matched PMC summaries for the config lines (every config
# line carries traffic): per config a rocprofv3 kernel trace of the bench
# command, separate FETCH_SIZE / WRITE_SIZE passes, scripts/pmc_summary.py ->
# profiles/${ROUND}_pmc_<config>.json.  EV = events per push (micro-batch),
# PUSHES = pushes in the trace run (calibration + warmup + steps).
#   ROUND=r06 CFGS="W2-length W2-time" bash scripts/gpu_profile_configs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
R=${ROUND:-r06}
for CFG in ${CFGS:-P3}; do
  case $CFG in
    P3|P3-dense) EV=50000896; PUSHES=8; STEPS="--steps 2 --warmup 1" ;;
    W2-length|W2-time) EV=50000896; PUSHES=6; STEPS="--steps 2 --warmup 1" ;;
    S4P-seqplus) EV=10000000; PUSHES=4; STEPS="--steps 2 --warmup 1" ;;
    M5) EV=10000384; PUSHES=30; STEPS="--steps 2 --warmup 1" ;;
    *) EV=1000000; PUSHES=4; STEPS="--steps 2 --warmup 1" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${R}_trace_${CFG} -o k -- python3 -u bench.py \
      --config $CFG $STEPS --cpu-sample 0 > gpurun_out/${R}_trace_${CFG}.log 2>&1
  rc=$?; echo "$CFG trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $C -f csv -d gpurun_out/${R}_pmc_${CFG}_$C -o k -- python3 -u bench.py \
        --config $CFG $STEPS --cpu-sample 0 > gpurun_out/${R}_pmc_${CFG}_$C.log 2>&1
    rc=$?; echo "$CFG pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/pmc_summary.py --trace gpurun_out/${R}_trace_${CFG}/k_kernel_trace.csv \
      --fetch gpurun_out/${R}_pmc_${CFG}_FETCH_SIZE/k_counter_collection.csv \
      --write gpurun_out/${R}_pmc_${CFG}_WRITE_SIZE/k_counter_collection.csv --events $EV --pushes $PUSHES \
      --out gpurun_out/${R}_pmc_${CFG}.json | cut -c1-300 || exit 1
  cp gpurun_out/${R}_pmc_${CFG}.json profiles/
  cp gpurun_out/${R}_trace_${CFG}/k_kernel_stats.csv profiles/${R}_${CFG}_kernel_stats.csv
done
exit 0
