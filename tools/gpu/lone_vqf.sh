#!/bin/bash
# lone / small-batch VQF timings and their kernel breakdown (rocprofv3 kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${O:-lone}; mkdir -p $O
timeout -k 10 300 python tools/small_batch.py --kind 1 --leaves ${LEAVES:-1,8,64,256,512,768,1024} --reps 50 > $O/timing.log 2>&1 || { tail -20 $O/timing.log; exit 3; }
cat $O/timing.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
for L in 1 64; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof$L -o p --output-format csv -- python $GRAFT_REPO_ROOT/tools/small_batch.py --kind 1 --leaves $L --reps 50 > $GRAFT_REPO_ROOT/$O/prof$L.log 2>&1 || exit 5
echo "## leaves $L"; cut -d, -f1-8 $GRAFT_REPO_ROOT/$O/prof$L/p_kernel_stats.csv | cut -c1-200
done
