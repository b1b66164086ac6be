#!/bin/bash
# Radix sort tile-shape sweep (prebuilt by scripts/build_sortbench.sh); _E1/_E2
# binaries are timing experiments whose output is not sorted (bad > 0 expected).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sortbench.jsonl
: > $out
for b in bench_bin/sortbench_*; do
  timeout -k 5 60 $b 50000000 10000000 5 1 >> $out; rc=$?
  case $b in *_E0) [ $rc -eq 0 ] || { echo "FAIL $b rc=$rc"; exit 1; } ;; *) [ $rc -le 1 ] || exit 1 ;; esac
done
cat $out
export TMPDIR=/tmp
for e in 0 1 2; do
  timeout -k 5 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sb_prof_E$e -o sb -- bench_bin/sortbench_R24_B256_E$e \
      50000000 10000000 3 1 > gpurun_out/sb_prof_E$e.log 2>&1
  rc=$?; [ $rc -le 1 ] || { echo "rocprof E$e rc=$rc"; exit 1; }
done
