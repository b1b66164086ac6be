# lockstep walk diagnostics: parity tests, kernel stats and SQ counters on P3-dense
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lockstep.py > gpurun_out/ls_t2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ls_t2.log; [ $rc -eq 0 ] || exit $rc
for LS in 0 1; do
  SHD_LOCKSTEP=$LS timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ls_tr$LS -o k -- python3 -u bench.py --config P3-dense \
    --steps 1 --warmup 0 --cpu-sample 0 --events 50000000 > gpurun_out/ls_tr$LS.log 2>&1
  rc=$?; echo "trace $LS rc=$rc"; [ $rc -eq 0 ] || exit $rc
  SHD_LOCKSTEP=$LS timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
    -f csv -d gpurun_out/ls_sq$LS -o k -- python3 -u bench.py --config P3-dense --steps 1 --warmup 0 --cpu-sample 0 --events 50000000 > gpurun_out/ls_sq$LS.log 2>&1
  rc=$?; echo "sq $LS rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
