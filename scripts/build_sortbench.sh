#!/bin/bash
# Build sortbench variants (tile rounds x block size [x timing experiment]) into bench_bin/.
set -eu
cd "$(dirname "$0")/.."
mkdir -p bench_bin
rm -f bench_bin/sortbench_*
for v in "24 256 0" "24 256 1" "24 256 2" "16 512 0" "32 256 0"; do
  set -- $v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSHD_RS_ROUNDS=$1 -DSHD_RS_BLOCK=$2 \
    -DSHD_RS_EXP=$3 -x hip scripts/sortbench.hip -o bench_bin/sortbench_R$1_B$2_E$3 &
done
wait
ls bench_bin
