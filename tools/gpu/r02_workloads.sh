#!/bin/bash
# Full-size bench lines for every BASELINE workload (one GPU): outputs in gpurun_out/$O
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/${O:-wl}; mkdir -p $O
for w in ${WORKLOADS:-vqf12 probe10 probe_vqf12 bloom12}; do
  timeout -k 10 400 python bench.py --workload $w > $O/bench_$w.log 2>&1 || exit 3
  tail -n 1 $O/bench_$w.log | cut -c1-400
done
if [ -n "$BIG" ]; then
  timeout -k 10 600 python bench.py --workload bloom12 --total-keys 1000000000 --no-e2e > $O/bench_bloom12_1B.log 2>&1 || exit 4
  tail -n 1 $O/bench_bloom12_1B.log | cut -c1-400
fi
