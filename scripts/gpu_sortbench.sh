#!/bin/bash
# Radix sort tile-shape sweep (prebuilt by scripts/build_sortbench.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sortbench.jsonl
: > $out
for b in bench_bin/sortbench_*; do
  for tri in 1 0; do
    timeout -k 5 60 $b 50000000 10000000 5 $tri >> $out || { echo "FAIL $b $tri rc=$?"; exit 1; }
  done
  SHD_RS_NOXCD=1 timeout -k 5 60 $b 50000000 10000000 5 1 >> $out || { echo "FAIL $b noxcd"; exit 1; }
done
cat $out
