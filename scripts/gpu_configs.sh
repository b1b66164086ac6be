#!/bin/bash
# Config lines, each with parity_prefix (device == oracle on the
# stream's first CPU-sample events) and the oracle's cpu_baseline:
#   CONFIGS="P1 P3-dense ..." TAG=r03 bash scripts/gpu_configs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
for c in ${CONFIGS:-P1 P3-dense W2-length W2-time S4-seq S4-seq14 S4-seqplus S4-or S4-and S4-not S4P-seqplus}; do
  case $c in
    P3-dense) CPU=1000000 ;;
    W2-*) CPU=1000000 ;;
    *) CPU=${CPU_SAMPLE:-1000000} ;;
  esac
  timeout -k 10 420 python3 -u bench.py --config $c --cpu-sample $CPU > gpurun_out/cfg_${TAG}_$c.json 2> gpurun_out/cfg_${TAG}_$c.err
  rc=$?; echo "== $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e6,1), 'M ev/s', d['ms_per_step'], d.get('stage_ms_per_step'), (d.get('cpu_baseline') or {}).get('value'), d.get('parity_prefix'), (d.get('derived_check') or {}).get('equal'))" gpurun_out/cfg_${TAG}_$c.json
done
if [ -n "${M5_EVENTS:-}" ]; then
  timeout -k 10 600 python3 -u bench.py --config M5 --events $M5_EVENTS --steps 1 --warmup 1 --cpu-sample 20000 > gpurun_out/cfg_${TAG}_M5.json 2> gpurun_out/cfg_${TAG}_M5.err
  rc=$?; echo "== M5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['query_events_per_s'], d['ms_per_step'], d.get('parity_prefix'))" gpurun_out/cfg_${TAG}_M5.json
fi
exit 0
