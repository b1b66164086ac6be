#!/bin/bash
# End-to-end InputHandler lines (bench.py --e2e) for P3 and W2-length.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for C in ${CFGS:-P3 W2-length}; do
  timeout -k 10 600 python3 -u bench.py --e2e --config $C > gpurun_out/r06_e2e_$C.json 2> gpurun_out/r06_e2e_$C.err || { tail -5 gpurun_out/r06_e2e_$C.err; exit 1; }
  tail -c 900 gpurun_out/r06_e2e_$C.json; echo
done
exit 0
