#!/bin/bash
# small-batch curve with per-kernel times (rocprofv3); outputs in gpurun_out/$O
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/${O:-small}; mkdir -p $O
for k in ${KINDS:-0 1}; do
  timeout -k 10 300 python tools/small_batch.py --kind $k --leaves ${CL:-1,8,64,256,1024,2048} > $O/curve_k$k.log 2>&1 || exit 2
  cat $O/curve_k$k.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_k$k -o run -- python tools/small_batch.py --kind $k --reps 20 --leaves $PL > $O/prof_k$k.log 2>&1 || exit 3
done
find $O -name "*kernel_stats.csv" | head
