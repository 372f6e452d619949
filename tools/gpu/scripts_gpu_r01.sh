#!/bin/bash
# round-1 GPU measurement script (run via gpurun); every GPU step has its own time limit
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_bloom10.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --workload vqf12 --no-e2e > gpurun_out/bench_vqf12.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --workload probe10 --no-cpu-baseline > gpurun_out/bench_probe10.log 2>&1 || exit 3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $GRAFT_REPO_ROOT/gpurun_out/prof_bloom10 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/gpurun_out/prof_bloom10.log 2>&1 || exit 4
