#!/bin/bash
# LeafBatcher VQF / Bloom from 16 and 32 threads: batch size and linger sweep
set -o pipefail
O=gpurun_out/r05/leaf; mkdir -p $O
B=$O/bench.txt
LB=/tmp/leaf_bench_$$
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude -o $LB tools/leaf_bench.cpp -Lturtle_kv_amd -ltkv_amq -Wl,-rpath,$PWD/turtle_kv_amd || exit 2
for kind in 1 0; do
  for cfg in "16 8 20" "16 16 20" "16 16 0" "16 16 50" "32 16 20" "32 32 20" "32 32 50"; do
    set -- $cfg
    timeout -k 10 60 $LB $1 2048 16384 $kind 1 $2 $3 >> $B 2>&1 || exit 3
  done
done
grep -v amdgpu.ids $B
