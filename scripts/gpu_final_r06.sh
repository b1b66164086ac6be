#!/bin/bash
# Round-6 closing lines: the headline P3 bench line (driver command, defaults),
# smoke, and the end-to-end InputHandler lines (bench.py --e2e) for P3 and W2-length.
#   ROUND=r06b bash scripts/gpu_final_r06.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${ROUND:-r06}
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${R}_smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/${R}_bench_P3.json 2> gpurun_out/${R}_bench_P3.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${R}_bench_P3.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'G', d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic_ratio'], d['parity_prefix'])"
for C in P3 W2-length; do
  timeout -k 10 600 python3 -u bench.py --e2e --config $C > gpurun_out/${R}_e2e_$C.json 2> gpurun_out/${R}_e2e_$C.err || exit 1
  tail -c 700 gpurun_out/${R}_e2e_$C.json
done
exit 0
