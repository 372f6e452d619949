#!/bin/bash
# C++ mirror test, then per-leaf drop-in vs LeafBatcher (tools/leaf_bench.cpp)
set -e
O=gpurun_out/${O:-leafb}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_cpp_mirror.py -v -m gpu --timeout 150 --timeout-method thread > $O/t.log 2>&1
B=$O/bench.txt
for kind in 0 1; do for t in 8 16 32; do
  timeout -k 10 60 ./tools/leaf_bench $t 2048 16384 $kind 0 >> $B 2>&1
  timeout -k 10 60 ./tools/leaf_bench $t 2048 16384 $kind 1 >> $B 2>&1
done; done
timeout -k 10 60 ./tools/leaf_bench 32 2048 16384 0 1 16 20 >> $B 2>&1
timeout -k 10 60 ./tools/leaf_bench 16 4096 4096 0 0 >> $B 2>&1
timeout -k 10 60 ./tools/leaf_bench 16 4096 4096 0 1 >> $B 2>&1
timeout -k 10 60 ./tools/leaf_bench 16 4096 4096 0 1 16 20 >> $B 2>&1
