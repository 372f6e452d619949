#!/bin/bash
# small-batch curve for experiment libraries tools/exp/libtkv_amq_<L>.so (LIBS="A B", KIND)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab_curve
for l in ${LIBS:-A B}; do
  TKV_AMQ_LIB=$GRAFT_REPO_ROOT/tools/exp/libtkv_amq_$l.so timeout -k 10 300 python tools/small_batch.py --kind ${KIND:-1} --leaves ${CL:-1,64,256,1024,6104} > gpurun_out/ab_curve/$l.log 2>&1 || exit 3
  echo "== $l"; grep kind gpurun_out/ab_curve/$l.log
done
