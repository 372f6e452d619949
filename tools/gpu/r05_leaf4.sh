#!/bin/bash
# LeafBatcher with one copy in and one copy out per batch: the C++ mirror test, then 16/32 callers
set -o pipefail
O=gpurun_out/r05/${TAG:-leaf5}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cpp_mirror.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
B=$O/bench.txt
LB=/tmp/leaf_bench_$$
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude -o $LB tools/leaf_bench.cpp -Lturtle_kv_amd -ltkv_amq -Wl,-rpath,$PWD/turtle_kv_amd || exit 3
for cfg in "16 1 8 60" "16 1 8 60" "16 1 8 100" "16 1 16 100" "32 1 16 60" "16 0 8 60" "32 0 16 60"; do
  set -- $cfg
  timeout -k 10 60 $LB $1 2048 16384 $2 1 $3 $4 >> $B 2>&1 || exit 4
done
grep -v amdgpu.ids $B | grep -A1 "threads" | grep -v "^--"
