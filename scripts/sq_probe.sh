#!/bin/bash
# SQ counters of one P3 bench step (instruction mix, waits, LDS bank conflicts),
# one --pmc pass per counter group.  Output: gpurun_out/${TAG}_sq_<n>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sq}
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G -f csv -d gpurun_out/${TAG}_sq_$i -o k -- python3 -u bench.py --config ${CFG:-P3} \
      --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/${TAG}_sq_$i.log 2>&1
  rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - gpurun_out/${TAG}_sq_1/k_counter_collection.csv gpurun_out/${TAG}_sq_2/k_counter_collection.csv <<'PY'
import csv, sys
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(float))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:48]
        if not any(x in k for x in ('scatter', 'k_ks_', 'forward', 'gather_list', 'k_prepare')):
            continue
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in agg.items():
    print(k, {c: '%.3g' % x for c, x in sorted(v.items())})
PY
