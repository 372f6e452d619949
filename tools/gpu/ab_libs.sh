#!/bin/bash
# A/B timing of library builds in tools/exp/ (LIBS="old new", W=workload), alternating runs
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  for l in ${LIBS:-old new}; do
    TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 200 python bench.py --workload ${W:-vqf12} \
      --no-cpu-baseline --no-e2e --no-verify --steps 20 > gpurun_out/ab_$l.log 2>&1 || exit 3
    echo "$l: $(python -c "import json;l=json.loads(open('gpurun_out/ab_$l.log').read().strip().splitlines()[-1]);print(l['value'], l['roofline']['kernel_ms'])")"
  done
done
