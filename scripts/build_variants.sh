#!/bin/bash
# Timing-experiment builds of libsiddhi_hip.so into bench_bin/ (used with
# SHD_LIB=bench_bin/<name>.so python bench.py ...).  Usage: build_variants.sh NAME "-DFLAG=1 ..."
set -eu
cd "$(dirname "$0")/../siddhi_amd/csrc"
name=$1; flags=$2
out=../../bench_bin/obj_$name
mkdir -p $out
for f in shd_api.cpp primitives.hip engine_pattern.hip engine_single.hip engine_nfa.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 $flags -std=c++17 -fPIC -ffp-contract=off -x hip -c $f -o $out/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../bench_bin/$name.so $out/*.o
rm -rf $out
