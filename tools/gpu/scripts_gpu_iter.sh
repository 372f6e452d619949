#!/bin/bash
# quick iteration: GPU parity tests + benches (+ optional rocprof of a workload)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 2
for w in ${WORKLOADS:-bloom10 vqf12 probe10}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --workload $w --no-e2e --no-cpu-baseline > gpurun_out/bench_$w.log 2>&1 || exit 3
done
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/prof_$PROF -o run --output-format csv -- python3 $R/bench.py --workload $PROF --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_$PROF.log 2>&1 || exit 4
fi
