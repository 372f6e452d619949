#!/bin/bash
# LeafBatcher timeline: HIP API, copies and kernels of 16 callers building VQF leaves
set -o pipefail
O=gpurun_out/r05/leaftrace; mkdir -p $O
LB=/tmp/leaf_bench_$$
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude -o $LB tools/leaf_bench.cpp -Lturtle_kv_amd -ltkv_amq -Wl,-rpath,$PWD/turtle_kv_amd || exit 2
export TMPDIR=/tmp
timeout -k 10 120 $LB 16 1024 16384 1 1 8 20 > $O/plain.txt 2>&1 || exit 3
timeout -k 10 240 rocprofv3 --runtime-trace --stats -d $O/trace -o run --output-format csv -- $LB 16 1024 16384 1 1 8 20 > $O/traced.txt 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu $O/plain.txt; ls $O/trace; exit $rc
