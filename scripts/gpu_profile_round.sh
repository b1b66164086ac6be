#!/bin/bash
# Round profile set for the P3 bench (copy the outputs into profiles/ afterwards):
#   1. rocprofv3 --kernel-trace --stats of the default bench command (csv)
#   2. separate --pmc FETCH_SIZE / WRITE_SIZE passes over one default-size push
#   3. scripts/pmc_summary.py -> per-stage HBM bytes (gfx950 corrections)
#   4. the default bench line (roofline.traffic read from step 3, cpu_baseline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
R=${ROUND:-r01}
CFG=${CFG:-P3}
EV=${EV:-50000000}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${R}_trace_${CFG} -o k -- python3 -u bench.py --config $CFG \
    --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/${R}_trace_${CFG}.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C -f csv -d gpurun_out/${R}_pmc_${CFG}_$C -o k -- python3 -u bench.py --config $CFG \
      --steps 1 --warmup 0 --cpu-sample 0 --events $EV > gpurun_out/${R}_pmc_${CFG}_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py --trace gpurun_out/${R}_trace_${CFG}/k_kernel_trace.csv \
    --fetch gpurun_out/${R}_pmc_${CFG}_FETCH_SIZE/k_counter_collection.csv \
    --write gpurun_out/${R}_pmc_${CFG}_WRITE_SIZE/k_counter_collection.csv --events $EV --pushes ${PUSHES:-8} \
    --out gpurun_out/${R}_pmc_${CFG}.json > /dev/null || exit 1
cp gpurun_out/${R}_pmc_${CFG}.json profiles/
timeout -k 10 600 python3 -u bench.py --config $CFG > gpurun_out/${R}_bench_${CFG}.json 2> gpurun_out/${R}_bench_${CFG}.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/${R}_bench_${CFG}.json
exit $rc
