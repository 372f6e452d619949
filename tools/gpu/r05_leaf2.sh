#!/bin/bash
# LeafBatcher VQF from 16 callers: longer lingers
set -o pipefail
O=gpurun_out/r05/leaf3; mkdir -p $O
B=$O/bench.txt
LB=/tmp/leaf_bench_$$
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude -o $LB tools/leaf_bench.cpp -Lturtle_kv_amd -ltkv_amq -Wl,-rpath,$PWD/turtle_kv_amd || exit 2
for cfg in "16 8 40" "16 8 60" "16 8 80" "16 6 60" "16 4 60" "16 6 40" "16 8 60"; do
  set -- $cfg
  timeout -k 10 60 $LB $1 2048 16384 1 1 $2 $3 >> $B 2>&1 || exit 3
done
grep -v amdgpu.ids $B | grep -A1 "16 threads"
