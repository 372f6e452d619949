#!/bin/bash
# window-path Bloom: parity tests, then timings of big-leaf batches (+ kernel stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${O:-win}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py -x -v -k "window or bloom" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/small_batch.py --leaf-keys 200000 --bpk 12 --leaves 1,8,70,256,512 --reps 20 > $O/big200k_12.log 2>&1 || exit 3
cat $O/big200k_12.log
timeout -k 10 300 python tools/small_batch.py --leaf-keys 140000 --bpk 10 --leaves 1,70,512 --reps 20 > $O/big140k_10.log 2>&1 || exit 4
cat $O/big140k_10.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o win -- python $GRAFT_REPO_ROOT/tools/small_batch.py --leaf-keys 200000 --bpk 12 --leaves 70 --reps 20 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 5
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -12
