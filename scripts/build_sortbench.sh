#!/bin/bash
# Build sortbench variants (tile rounds x block size) into bench_bin/.
set -eu
cd "$(dirname "$0")/.."
mkdir -p bench_bin
for v in "16 256" "8 256" "24 256" "8 512" "12 512" "16 512"; do
  set -- $v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSHD_RS_ROUNDS=$1 -DSHD_RS_BLOCK=$2 \
    -x hip scripts/sortbench.hip -o bench_bin/sortbench_R$1_B$2 &
done
wait
ls bench_bin
