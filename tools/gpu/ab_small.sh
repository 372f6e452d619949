#!/bin/bash
# Small-batch curve for library builds in tools/exp/ (LIBS="e0 e1 ..."), KIND, LEAVES
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/${O:-absmall}; mkdir -p $O
for l in ${LIBS:-old new}; do
  TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 200 python tools/small_batch.py --kind ${KIND:-1} \
    --leaves ${LEAVES:-1,64,1024,6104} --reps ${REPS:-20} > $O/small_$l.log 2>&1 || exit 4
  echo "== $l"; grep kind $O/small_$l.log
done
