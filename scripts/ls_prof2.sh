# walk kernel counters on P3-dense (lockstep default): SQ issue mix, then L2 hits
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
  -f csv -d gpurun_out/ls2_sq -o k -- python3 -u bench.py --config P3-dense --steps 1 --warmup 0 --cpu-sample 0 --events 50000000 > gpurun_out/ls2_sq.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM TCC_HIT_sum TCC_MISS_sum \
  -f csv -d gpurun_out/ls2_mem -o k -- python3 -u bench.py --config P3-dense --steps 1 --warmup 0 --cpu-sample 0 --events 50000000 > gpurun_out/ls2_mem.log 2>&1
rc=$?; echo "mem rc=$rc"; exit $rc
