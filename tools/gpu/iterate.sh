#!/bin/bash
# iteration: the parity tests that touch this round's kernels, then timings (+ kernel stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${O:-it}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -v -k "${K:-window or bloom or vqf}" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
rm -f $O/timing.log
while IFS= read -r args; do
  [ -z "$args" ] && continue
  echo "## $args" >> $O/timing.log
  timeout -k 10 300 python tools/small_batch.py $args --reps 20 2>&1 | grep -v amdgpu.ids >> $O/timing.log || exit 3
done <<'ARGS'
--leaf-keys 200000 --bpk 12 --leaves 70,512
--leaf-keys 200000 --bpk 12 --leaves 70,512 --no-ws
--leaf-keys 140000 --bpk 10 --leaves 70,512
--leaf-keys 140000 --bpk 10 --leaves 1,8,70,512 --no-ws
--kind 1 --key-bytes 0 --leaves 1,768,1024,2048,6104
--kind 1 --key-bytes 16 --leaves 1,768,6104
--kind 1 --key-bytes 24 --leaves 6104
--kind 0 --key-bytes 0 --leaves 6104
ARGS
cat $O/timing.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o win --output-format csv -- python $GRAFT_REPO_ROOT/tools/small_batch.py --leaf-keys 200000 --bpk 12 --leaves 512 --reps 20 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 5
cut -d, -f1-4 $GRAFT_REPO_ROOT/$O/prof/win_kernel_stats.csv | cut -c1-150
