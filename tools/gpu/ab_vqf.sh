#!/bin/bash
# VQF A/B of library builds in tools/exp/ (LIBS="old new"): parity tests of the last library,
# full-batch bench (vqf12) and the small-batch curve, alternating runs.  Outputs: gpurun_out/$O
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/${O:-abvqf}; mkdir -p $O
LIBS=${LIBS:-old new}
last=${LIBS##* }
TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$last.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu \
  -k "${TESTS:-vqf or VQF}" --timeout 200 --timeout-method thread > $O/tests_$last.log 2>&1 || { tail -20 $O/tests_$last.log; exit 2; }
tail -1 $O/tests_$last.log
for rep in 1 2; do
  for l in $LIBS; do
    TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 200 python bench.py --workload ${W:-vqf12} \
      --no-cpu-baseline --no-e2e --no-verify --steps 20 > $O/bench_${l}_$rep.log 2>&1 || exit 3
    echo "$l: $(python -c "import json;l=json.loads(open('$O/bench_${l}_$rep.log').read().strip().splitlines()[-1]);print(l['value'], l['roofline']['kernel_ms'])")"
  done
done
for l in $LIBS; do
  TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 200 python tools/small_batch.py --kind 1 \
    --leaves ${LEAVES:-1,8,64,256,1024} > $O/small_$l.log 2>&1 || exit 4
  echo "== $l"; grep kind $O/small_$l.log
done
